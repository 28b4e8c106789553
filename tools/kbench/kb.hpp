// kb.hpp — the interface between tools/kbench/kbench.cpp and its kernels (kb_kernels.hip).
// kbench compiles the library's device code (csrc/kernels_dev.hpp) with launchers of its own, so
// the experiments below never reach libnttmul.so: the rejected kernels (k_rows_w4, k_rows_pipe,
// k_rows_ab, k_mp_persist) and the wrong-result pricing variants (KB_ABL_* flags, kb_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "launch.hpp"

namespace kb {

struct Conf {
  int mp_lag = 0;            // n > 4096: > 0 = one persistent launch (k_mp_persist) with this
                             // many steps between a polynomial's column, row and inverse tasks
  void *mp_stats = nullptr;  // NTTMUL_MP_STATS builds: 9 u64 task statistics
  int mp_phase = -1;         // n > 4096: -1 all three passes, 0 only the forward column pass,
                             // 1 only the row pass, 2 only the inverse column pass
  int rows_lds_extra = 0;    // n > 4096: dynamic LDS bytes added to each row-pass workgroup (caps
                             // the row pass's workgroups per CU, leaving room for column waves)
  int pipe_per_wave = 0;     // n = 1024, q < 2^31: > 0 = k_rows_pipe with this many products per
                             // wave; -1 = k_rows_w4; -2 = k_rows_ab; 0 = k_rows (the library's)
};

// Bytes of the ticket / counter words k_mp_persist needs for `batch` polynomials (scr[3]).
inline size_t mp_sync_bytes(size_t batch) { return (2 * batch + 2) * sizeof(unsigned); }

// c = a * b as launch_polymul, for the kernel set this binary was built with (KB_SET 1: u32
// words, q < 2^31, n <= 4096; KB_SET 2: 64-bit words, n = 65536).  scr[3]: mp_sync_bytes.
hipError_t launch(const nttmul::LaunchTables &T, const Conf &C, const void *a, const void *b,
                  void *c, size_t batch, int io_bits, void **scr, hipStream_t s);
hipError_t fill(void *a, void *b, uint32_t logn, uint64_t q, uint64_t seed, size_t count,
                int io_bits, hipStream_t s);
const char *set_name();

}  // namespace kb
