// kernels.hip — the library's launchers (the host side of include/nttmul.h's device calls): which
// kernel of kernels_dev.hpp runs for which (n, q, word size, batch), with what launch shape.
// This is the translation unit of libnttmul.so's kernels; the tools/kbench timing binaries
// include kernels_dev.hpp with launchers of their own and never compile this file.
#if defined(NTTMUL_HOOK_ROWS_LD) || defined(NTTMUL_HOOK_ROWS_ST) || defined(NTTMUL_HOOK_ROWS_INPUT) || \
    defined(NTTMUL_HOOK_ROWS_OUTPUT) || defined(NTTMUL_HOOK_XCHG) || defined(NTTMUL_HOOK_COLS_LD) || \
    defined(NTTMUL_HOOK_COLS_ST) || defined(NTTMUL_HOOK_TW) || defined(NTTMUL_HOOK_PRIO0)
#error "NTTMUL_HOOK_* are tools/kbench instrumentation points (wrong-result pricing builds), not library switches"
#endif
#include "kernels_dev.hpp"

namespace nttmul {

// Fused single-launch product, n = 2^logn <= 4096.
template <class A, class IO>
static hipError_t fused(const LaunchTables &T, const void *a, const void *b, void *c,
                        size_t batch, hipStream_t s) {
  const KParams<A> P = product_params<A>(T);
  switch (T.logn) {
    case 8: return launch_rows<A, IO, IO, 8, 0>(P, a, b, c, batch, s);
    case 9: return launch_rows<A, IO, IO, 9, 0>(P, a, b, c, batch, s);
    case 10: return launch_rows<A, IO, IO, 10, 0>(P, a, b, c, batch, s);
    case 11: return launch_rows<A, IO, IO, 11, 0>(P, a, b, c, batch, s);
    case 12: return launch_rows<A, IO, IO, 12, 0>(P, a, b, c, batch, s);
    default: return hipErrorInvalidValue;
  }
}

// Multi-pass product, n = 2^logn in (4096, 65536]: rows of 4096, L1 = logn - 12 column stages.
template <class A, class IO, int L1, int LOGS = 12>
static hipError_t multipass_l1(const LaunchTables &T, const void *a, const void *b, void *c,
                               size_t batch, void *ta, void *tb, void *tc, hipStream_t s) {
  using W = typename A::word;
  const KParams<A> P = product_params<A>(T);
  const size_t cols = batch << LOGS;
  const unsigned cblocks = (unsigned)((cols + 255) / 256);
  if (tl_describe) {
    const std::string args = std::string(AName<A>::v) + "," + word_name<IO>() + "," +
                             std::to_string(L1);
    describe_add("k_cols_fwd<" + args + ">");
    (void)launch_rows<A, W, W, LOGS, L1>(P, ta, tb, tc, batch << L1, s);
    describe_add("k_cols_inv<" + args + ">");
    return hipSuccess;
  }
  hipLaunchKernelGGL((k_cols_fwd<A, IO, L1>), dim3(cblocks), dim3(256), 0, s, P, (const IO *)a,
                     (const IO *)b, (W *)ta, (W *)tb, batch, LOGS);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = launch_rows<A, W, W, LOGS, L1>(P, ta, tb, tc, batch << L1, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_cols_inv<A, IO, L1>), dim3(cblocks), dim3(256), 0, s, P,
                     (const W *)tc, (IO *)c, batch, LOGS);
  return hipGetLastError();
}


// Multi-pass product of the square split, n = 65536 = 256 x 256 (64-bit words, NTTMUL_C5_SQ):
// k_cols8 forward (global stages 0..7 of a and b), the row pass k_rows<..., 8, 8> (stages 8..15,
// base multiplication, inverse stages 15..8 of 256-coefficient rows), k_cols8 inverse.
template <class A, class IO>
static hipError_t multipass_sq(const LaunchTables &T, const void *a, const void *b, void *c,
                               size_t batch, void *ta, void *tb, void *tc, hipStream_t s) {
  using W = typename A::word;
  const KParams<A> P = product_params<A>(T);
  const size_t groups = batch * 16;  // 16 workgroups of 16 columns per polynomial
  if (tl_describe) {
    const std::string args = std::string(AName<A>::v) + "," + word_name<IO>();
    describe_add("k_cols8<" + args + ",fwd>");
    (void)launch_rows<A, W, W, 8, 8>(P, ta, tb, tc, batch << 8, s);
    describe_add("k_cols8<" + args + ",inv>");
    return hipSuccess;
  }
  if (groups == 0) return hipSuccess;
  hipLaunchKernelGGL((k_cols8<A, IO, W, 0>), dim3((unsigned)groups), dim3(256), 0, s, P,
                     (const IO *)a, (const IO *)b, (W *)ta, (W *)tb, groups);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = launch_rows<A, W, W, 8, 8>(P, ta, tb, tc, batch << 8, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_cols8<A, W, IO, 1>), dim3((unsigned)groups), dim3(256), 0, s, P,
                     (const W *)tc, (const W *)nullptr, (IO *)c, (IO *)nullptr, groups);
  return hipGetLastError();
}

template <class A, class IO>
static hipError_t multipass(const LaunchTables &T, const void *a, const void *b, void *c,
                            size_t batch, void **scr, hipStream_t s) {
  if constexpr (sizeof(typename A::word) == 8 && NTTMUL_C5_SQ) {
    if (T.logn == 16) return multipass_sq<A, IO>(T, a, b, c, batch, scr[0], scr[1], scr[2], s);
  }
  switch (T.logn) {
    case 13: return multipass_l1<A, IO, 1>(T, a, b, c, batch, scr[0], scr[1], scr[2], s);
    case 14: return multipass_l1<A, IO, 2>(T, a, b, c, batch, scr[0], scr[1], scr[2], s);
    case 15: return multipass_l1<A, IO, 3>(T, a, b, c, batch, scr[0], scr[1], scr[2], s);
    case 16:
      if (NTTMUL_SPLIT16 == 5)  // 32 x 2048: one more stage in the (HBM-bound) column passes
        return multipass_l1<A, IO, 5, 11>(T, a, b, c, batch, scr[0], scr[1], scr[2], s);
      return multipass_l1<A, IO, 4>(T, a, b, c, batch, scr[0], scr[1], scr[2], s);
    default: return hipErrorInvalidValue;
  }
}

template <class A>
static hipError_t polymul_io(const LaunchTables &T, const void *a, const void *b, void *c,
                             size_t batch, int io_bits, void **scr, hipStream_t s) {
  const bool big = T.logn > 12;
  if constexpr (std::is_same<A, Arith32P>::value) {  // D = 3 blocks at n = 4096 (Arith32P3)
    if (T.logn == 12 && p3_fold_ok(T.q)) {
      const KParams<Arith32P3> P = product_params<Arith32P3>(T);
      return io_bits == 64 ? launch_rows<Arith32P3, uint64_t, uint64_t, 12, 0>(P, a, b, c, batch, s)
                           : launch_rows<Arith32P3, uint32_t, uint32_t, 12, 0>(P, a, b, c, batch, s);
    }
  }
  if (io_bits == 64)
    return big ? multipass<A, uint64_t>(T, a, b, c, batch, scr, s)
               : fused<A, uint64_t>(T, a, b, c, batch, s);
  return big ? multipass<A, uint32_t>(T, a, b, c, batch, scr, s)
             : fused<A, uint32_t>(T, a, b, c, batch, s);
}

static hipError_t launch_polymul_(const LaunchTables &T, const void *a, const void *b, void *c,
                                  size_t batch, int io_bits, void **scr, hipStream_t s);
hipError_t launch_polymul(const LaunchTables &T, const void *a, const void *b, void *c,
                          size_t batch, int io_bits, void **scr, hipStream_t s) {
  const int prev = tl_prio_cus, prev_mode = tl_prio_mode;
  tl_prio_cus = T.prio_ok ? T.cus : 0;
  tl_prio_mode = T.prio;
  const hipError_t e = launch_polymul_(T, a, b, c, batch, io_bits, scr, s);
  tl_prio_cus = prev;
  tl_prio_mode = prev_mode;
  return e;
}
static hipError_t launch_polymul_(const LaunchTables &T, const void *a, const void *b, void *c,
                                  size_t batch, int io_bits, void **scr, hipStream_t s) {
  if (T.word_bits == 32) {  // 64-bit storage of a q < 2^32 product: same 32-bit arithmetic
    switch (a32_kind(T.q)) {
      case A32Kind::Harvey: return polymul_io<Arith32H>(T, a, b, c, batch, io_bits, scr, s);
      case A32Kind::Wide: return polymul_io<Arith32W>(T, a, b, c, batch, io_bits, scr, s);
      case A32Kind::Plantard: return polymul_io<Arith32P>(T, a, b, c, batch, io_bits, scr, s);
      case A32Kind::Mont: return polymul_io<Arith32>(T, a, b, c, batch, io_bits, scr, s);
    }
  }
  return polymul_io<Arith64>(T, a, b, c, batch, io_bits, scr, s);
}

hipError_t launch_server(const LaunchTables &T, const ServerReq *req, ServerBox *box,
                         unsigned long long idle_ticks, unsigned long long life_ticks,
                         hipStream_t s) {
  const size_t pairs = T.tw_bytes / sizeof(TwPair<uint32_t>);
  if (T.word_bits != 32 || a32_kind(T.q) != A32Kind::Plantard || T.logn < 8 || T.logn > 10 ||
      pairs > (1u << T.logn))
    return hipErrorNotSupported;
  const KParams<Arith32P> P = product_params<Arith32P>(T);
  const unsigned tp = (unsigned)pairs;
  switch (T.logn) {
    case 8: hipLaunchKernelGGL((k_server<Arith32P, 8>), dim3(1), dim3(512), 0, s, P, req, box, tp, idle_ticks, life_ticks); break;
    case 9: hipLaunchKernelGGL((k_server<Arith32P, 9>), dim3(1), dim3(64), 0, s, P, req, box, tp, idle_ticks, life_ticks); break;
    default: hipLaunchKernelGGL((k_server<Arith32P, 10>), dim3(1), dim3(128), 0, s, P, req, box, tp, idle_ticks, life_ticks); break;
  }
  return hipGetLastError();
}

hipError_t describe_polymul(const LaunchTables &T, int io_bits, size_t batch, std::string *out) {
  out->clear();
  void *scr[3] = {nullptr, nullptr, nullptr};
  tl_describe = out;
  const hipError_t e = launch_polymul(T, nullptr, nullptr, nullptr, batch ? batch : (size_t)1 << 24,
                                      io_bits, scr, nullptr);
  tl_describe = nullptr;
  return e;
}

template <class A, class TIn, class TOut, int LOGS, int L1, int DIR>
static hipError_t launch_xform_rows(const KParams<A> &P, const void *in, void *out, size_t units,
                                    hipStream_t s) {
  constexpr int PB = 256 / ((1 << LOGS) / 16) * xform_upg<A, L1, DIR>();
  const size_t blocks = (units + PB - 1) / PB;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((k_xform<A, TIn, TOut, LOGS, L1, DIR>), dim3((unsigned)blocks), dim3(256), 0,
                     s, P, (const TIn *)in, (TOut *)out, units);
  return hipGetLastError();
}

// KParams for the standalone inverse: scale by n^-1 only (no Montgomery factor)
template <class A>
static KParams<A> inverse_params(const LaunchTables &T) {
  KParams<A> P = make_params<A>(T);
  P.f = (typename A::word)T.fi; P.fs = (typename A::word)T.fis;
  P.wf = (typename A::word)T.wfi; P.wfs = (typename A::word)T.wfis;
  return P;
}

template <class A, class IO, int DIR>
static hipError_t xform_fused(const LaunchTables &T, const void *in, void *out, size_t batch,
                              hipStream_t s) {
  const KParams<A> P = DIR == 0 ? make_params<A>(T) : inverse_params<A>(T);
  switch (T.logn) {
    case 8: return launch_xform_rows<A, IO, IO, 8, 0, DIR>(P, in, out, batch, s);
    case 9: return launch_xform_rows<A, IO, IO, 9, 0, DIR>(P, in, out, batch, s);
    case 10: return launch_xform_rows<A, IO, IO, 10, 0, DIR>(P, in, out, batch, s);
    case 11: return launch_xform_rows<A, IO, IO, 11, 0, DIR>(P, in, out, batch, s);
    case 12: return launch_xform_rows<A, IO, IO, 12, 0, DIR>(P, in, out, batch, s);
    default: return hipErrorInvalidValue;
  }
}

template <class A, class IO, int L1, int DIR>
static hipError_t xform_multipass_l1(const LaunchTables &T, const void *in, void *out,
                                     size_t batch, void **scr, hipStream_t s) {
  using W = typename A::word;
  constexpr int LOGS = 12;
  const size_t cols = batch << LOGS;
  const unsigned cblocks = (unsigned)((cols + 255) / 256);
  if (DIR == 0) {
    const KParams<A> P = make_params<A>(T);
    hipLaunchKernelGGL((k_cols_fwd<A, IO, L1, 1>), dim3(cblocks), dim3(256), 0, s, P,
                       (const IO *)in, (const IO *)nullptr, (W *)scr[0], (W *)nullptr, batch,
                       LOGS);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_xform_rows<A, W, IO, LOGS, L1, 0>(P, scr[0], out, batch << L1, s);
  }
  const KParams<A> P = inverse_params<A>(T);
  hipError_t e = launch_xform_rows<A, IO, W, LOGS, L1, 1>(P, in, scr[0], batch << L1, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_cols_inv<A, IO, L1>), dim3(cblocks), dim3(256), 0, s, P,
                     (const W *)scr[0], (IO *)out, batch, LOGS);
  return hipGetLastError();
}

// Standalone transforms of the square split (64-bit words at n = 65536, NTTMUL_C5_SQ, as the
// product): forward = k_cols8 on one polynomial (tiled scratch) + the 256-coefficient row pass
// (k_xform<..., 8, 8, 0>); inverse = the row pass into the tiled scratch + k_cols8 inverse.
template <class A, class IO, int DIR>
static hipError_t xform_sq(const LaunchTables &T, const void *in, void *out, size_t batch,
                           void **scr, hipStream_t s) {
  using W = typename A::word;
  const size_t groups = batch * 16;
  if (groups == 0) return hipSuccess;
  if (DIR == 0) {
    const KParams<A> P = make_params<A>(T);
    hipLaunchKernelGGL((k_cols8<A, IO, W, 0, 1>), dim3((unsigned)groups), dim3(256), 0, s, P,
                       (const IO *)in, (const IO *)nullptr, (W *)scr[0], (W *)nullptr, groups);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_xform_rows<A, W, IO, 8, 8, 0>(P, scr[0], out, batch << 8, s);
  }
  const KParams<A> P = inverse_params<A>(T);
  hipError_t e = launch_xform_rows<A, IO, W, 8, 8, 1>(P, in, scr[0], batch << 8, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_cols8<A, W, IO, 1>), dim3((unsigned)groups), dim3(256), 0, s, P,
                     (const W *)scr[0], (const W *)nullptr, (IO *)out, (IO *)nullptr, groups);
  return hipGetLastError();
}

template <class A, class IO, int DIR>
static hipError_t xform_any(const LaunchTables &T, const void *in, void *out, size_t batch,
                            void **scr, hipStream_t s) {
  if constexpr (sizeof(typename A::word) == 8 && NTTMUL_C5_SQ) {
    if (T.logn == 16) return xform_sq<A, IO, DIR>(T, in, out, batch, scr, s);
  }
  switch (T.logn) {
    case 13: return xform_multipass_l1<A, IO, 1, DIR>(T, in, out, batch, scr, s);
    case 14: return xform_multipass_l1<A, IO, 2, DIR>(T, in, out, batch, scr, s);
    case 15: return xform_multipass_l1<A, IO, 3, DIR>(T, in, out, batch, scr, s);
    case 16: return xform_multipass_l1<A, IO, 4, DIR>(T, in, out, batch, scr, s);
    default: return xform_fused<A, IO, DIR>(T, in, out, batch, s);
  }
}

template <class A, int DIR>
static hipError_t xform_io(const LaunchTables &T, const void *in, void *out, size_t batch,
                           int io_bits, void **scr, hipStream_t s) {
  return io_bits == 64 ? xform_any<A, uint64_t, DIR>(T, in, out, batch, scr, s)
                       : xform_any<A, uint32_t, DIR>(T, in, out, batch, scr, s);
}

template <int DIR>
static hipError_t launch_xform_dir(const LaunchTables &T, const void *in, void *out, size_t batch,
                                   int io_bits, void **scr, hipStream_t s) {
  if (T.word_bits == 32) {
    switch (a32_kind(T.q)) {
      case A32Kind::Harvey: return xform_io<Arith32H, DIR>(T, in, out, batch, io_bits, scr, s);
      case A32Kind::Wide: return xform_io<Arith32W, DIR>(T, in, out, batch, io_bits, scr, s);
      case A32Kind::Plantard: return xform_io<Arith32P, DIR>(T, in, out, batch, io_bits, scr, s);
      case A32Kind::Mont: return xform_io<Arith32, DIR>(T, in, out, batch, io_bits, scr, s);
    }
  }
  return xform_io<Arith64, DIR>(T, in, out, batch, io_bits, scr, s);
}

hipError_t launch_xform(const LaunchTables &T, const void *in, void *out, size_t batch,
                        int io_bits, int inverse, void **scr, hipStream_t s) {
  return inverse ? launch_xform_dir<1>(T, in, out, batch, io_bits, scr, s)
                 : launch_xform_dir<0>(T, in, out, batch, io_bits, scr, s);
}

template <class A, class IO>
static hipError_t pointwise(const LaunchTables &T, const void *a, const void *b, void *c,
                            size_t total, hipStream_t s) {
  KParams<A> P = make_params<A>(T);
  P.f = (typename A::word)T.r2;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL((k_pointwise<A, IO>), dim3(blocks), dim3(256), 0, s, P, (const IO *)a,
                     (const IO *)b, (IO *)c, total);
  return hipGetLastError();
}

hipError_t launch_pointwise(const LaunchTables &T, const void *a, const void *b, void *c,
                            size_t batch, int io_bits, hipStream_t s) {
  const size_t total = batch << T.logn;
  if (!total) return hipSuccess;
  if (T.word_bits == 32 && T.q >= (1ull << 31))
    return io_bits == 64 ? pointwise<Arith32W, uint64_t>(T, a, b, c, total, s)
                         : pointwise<Arith32W, uint32_t>(T, a, b, c, total, s);
  if (T.word_bits == 32)  // Montgomery products only (no twiddle tables): Arith32 for q < 2^31
    return io_bits == 64 ? pointwise<Arith32, uint64_t>(T, a, b, c, total, s)
                         : pointwise<Arith32, uint32_t>(T, a, b, c, total, s);
  return io_bits == 64 ? pointwise<Arith64, uint64_t>(T, a, b, c, total, s)
                       : pointwise<Arith64, uint32_t>(T, a, b, c, total, s);
}

hipError_t launch_bitrev(const void *in, void *out, uint32_t logn, size_t batch, int io_bits,
                         hipStream_t s) {
  const size_t total = batch << logn;
  if (!total) return hipSuccess;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  if (in == out) {
    if (io_bits == 32)
      hipLaunchKernelGGL(k_bitrev_inplace<uint32_t>, dim3(blocks), dim3(256), 0, s, (uint32_t *)out,
                         logn, total);
    else
      hipLaunchKernelGGL(k_bitrev_inplace<uint64_t>, dim3(blocks), dim3(256), 0, s, (uint64_t *)out,
                         logn, total);
  } else if (io_bits == 32) {
    hipLaunchKernelGGL(k_bitrev<uint32_t>, dim3(blocks), dim3(256), 0, s, (const uint32_t *)in,
                       (uint32_t *)out, logn, total);
  } else {
    hipLaunchKernelGGL(k_bitrev<uint64_t>, dim3(blocks), dim3(256), 0, s, (const uint64_t *)in,
                       (uint64_t *)out, logn, total);
  }
  return hipGetLastError();
}

hipError_t launch_fill(void *a, void *b, uint32_t logn, uint64_t q, uint64_t seed, uint64_t p0,
                       size_t count, int io_bits, hipStream_t s) {
  const size_t total = count << logn;
  if (!total) return hipSuccess;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  if (io_bits == 32)
    hipLaunchKernelGGL(k_fill<uint32_t>, dim3(blocks), dim3(256), 0, s, (uint32_t *)a,
                       (uint32_t *)b, logn, q, seed, p0, total);
  else
    hipLaunchKernelGGL(k_fill<uint64_t>, dim3(blocks), dim3(256), 0, s, (uint64_t *)a,
                       (uint64_t *)b, logn, q, seed, p0, total);
  return hipGetLastError();
}

hipError_t launch_check_range(const void *a, const void *b, uint64_t q, size_t total, int io_bits,
                              int *bad, hipStream_t s) {
  if (!total) return hipSuccess;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  if (io_bits == 32)
    hipLaunchKernelGGL(k_check_range<uint32_t>, dim3(blocks), dim3(256), 0, s,
                       (const uint32_t *)a, (const uint32_t *)b, q, total, bad);
  else
    hipLaunchKernelGGL(k_check_range<uint64_t>, dim3(blocks), dim3(256), 0, s,
                       (const uint64_t *)a, (const uint64_t *)b, q, total, bad);
  return hipGetLastError();
}

}  // namespace nttmul