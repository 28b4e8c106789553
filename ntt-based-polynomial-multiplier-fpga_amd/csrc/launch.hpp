// launch.hpp — internal interface between the host runtime (nttmul.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace nttmul {

// Per-device view of a plan: what a launch needs (pointers are device memory).
struct LaunchTables {
  uint32_t logn;
  int word_bits;           // 32 -> Arith32H / Arith32 / Arith32W by q (q < 2^32), 64 -> Arith64
  uint64_t q, qinv_neg;    // -q^-1 mod 2^word_bits
  uint64_t f, fs, wf, wfs; // F = n^-1 R mod q and iw[1] F, as (value, companion) pairs
  uint64_t f4, f4s, wf4, wf4s; // 4 F and iw[1] 4 F: products with incomplete transforms (D = 2)
  uint64_t f8, f8s, wf8, wf8s; // 8 F and iw[1] 8 F (D = 3: Arith32P3)
  uint64_t fi, fis, wfi, wfis; // n^-1 and iw[1] n^-1 (standalone inverse), with companions
  uint64_t r2;             // R^2 mod q (standalone pointwise product)
  const void *fw, *iw;     // forward / inverse twiddle (value, companion) pairs, n entries
                           // (planner.cpp tw_pair: Shoup, or Montgomery form for Arith32)
  size_t tw_bytes = 0;     // bytes of each of fw, iw (2n pairs with Arith32's centred copies)
  int cus;                 // compute units of the device (launch-shape thresholds)
  int prio = 0;            // nttmul_params.issue_prio: -1 never, 0 automatic, 1 always
  int prio_ok = 1;         // 0: the previous product launch of this context went to another
                           // stream, so automatic mode keeps oldest-first issue (kernels.hip rows_prio)
};

// c = a * b for `batch` polynomials of n = 2^logn words of io_bits (32/64) each, on stream s.
// scr: three device buffers of batch * n words of word_bits, used only when n > 4096.
hipError_t launch_polymul(const LaunchTables &T, const void *a, const void *b, void *c,
                          size_t batch, int io_bits, void **scr, hipStream_t s);
// The kernels launch_polymul would launch for (T, io_bits), as "k_rows<Arith32P3,u32,u32,12,0>"
// (multi-pass: the three kernels joined by " + "); nothing is launched.
hipError_t describe_polymul(const LaunchTables &T, int io_bits, size_t batch, std::string *out);
// Standalone forward (inverse = 0) or inverse (inverse = 1) NTT of `batch` polynomials
// (SURVEY §8f row 1).  scr as for launch_polymul (only scr[0] is used).
hipError_t launch_xform(const LaunchTables &T, const void *in, void *out, size_t batch,
                        int io_bits, int inverse, void **scr, hipStream_t s);
// c = a * b mod q coefficient-wise over batch * n words.
hipError_t launch_pointwise(const LaunchTables &T, const void *a, const void *b, void *c,
                            size_t batch, int io_bits, hipStream_t s);
// Bit-reversal permutation of each of `batch` polynomials of 2^logn words (in == out: in place).
hipError_t launch_bitrev(const void *in, void *out, uint32_t logn, size_t batch, int io_bits,
                         hipStream_t s);
hipError_t launch_fill(void *a, void *b, uint32_t logn, uint64_t q, uint64_t seed, uint64_t p0,
                       size_t count, int io_bits, hipStream_t s);
// Mailbox of the small-transaction device server (k_server, nttmul.cpp Server), shared by one
// host caller and one resident kernel -- the MI355X form of the FPGA communicator's
// mode-3 GO + WaitForDoneAll polling (NTT_PCIECommunicationv2.c:83-107, 211-215).  The host sets
// c to kPending, writes a and b, then the go word (seq << 8) | count; the kernel (polling go)
// multiplies and writes c, and the request is complete when no word of c is kPending.  One word
// carries the sequence number and the product count, so the kernel learns both from one read;
// count 0 asks it to leave.
// done is the last go word already served: written by the host before each launch (the kernel
// starts from it) and, in the diagnostic build, by the kernel after its stamps.
// It has two halves, each crossing PCIe only as posted writes (round 4,
// tools/microbench/mailbox_latency.hip: a 256-word request's transport 2.6 us this way against
// 3.7 us with go, a and b in host memory, where every poll and operand load is a PCIe read):
// ServerReq (go, a, b: host -> device) lives in fine-grained device memory that the host maps
// through the large BAR (pinned host memory when the device offers no host mapping), ServerBox
// (c, done, stamps: device -> host) in pinned host memory.
struct ServerBox {
  static constexpr int kWords = 1024;            // per operand: n x count <= 1024 words
  static constexpr unsigned kStop = 0;           // count field of a stop request
  static constexpr uint32_t kPending = 0xFFFFFFFFu;  // no canonical coefficient (q < 2^31)
  alignas(128) uint32_t done;
  alignas(128) uint32_t c[kWords];
  // lib/libnttmul_diag.so: the last request's s_memrealtime stamps (request seen, a and b
  // loaded, product computed, c stored and released) and s_memtime around the product
  alignas(128) unsigned long long stamp[6];
};
struct ServerReq {
  alignas(128) uint32_t go;
  alignas(128) uint32_t a[ServerBox::kWords];
  alignas(128) uint32_t b[ServerBox::kWords];
};
// Launch the server for products of n = 2^logn <= 1024 u32 words (q < 2^31) on stream s; it
// leaves after idle_ticks of the 100 MHz clock without a request, after life_ticks in all, or
// on a stop request.  hipErrorNotSupported for other (n, q) or twiddle tables larger than the
// kernel's LDS copy (n pairs each).
hipError_t launch_server(const LaunchTables &T, const ServerReq *req, ServerBox *box,
                         unsigned long long idle_ticks, unsigned long long life_ticks,
                         hipStream_t s);

#ifdef NTTMUL_CLOCK_STAMPS
// lib/libnttmul_diag.so: the k_rows clock stamps of the last launch, 4 u64 per workgroup
// (entry memtime, entry realtime, end memtime, end realtime), workgroups 0 .. blocks - 1
hipError_t read_clock_stamps(void *dst, size_t blocks);
#endif
hipError_t launch_check_range(const void *a, const void *b, uint64_t q, size_t total, int io_bits,
                              int *bad, hipStream_t s);

}  // namespace nttmul
