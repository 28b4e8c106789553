// kb_kernels.hip — tools/kbench's kernels: the library's device code (csrc/kernels_dev.hpp) with
// launchers of kbench's own, the C2 / C5 experiments the library does not carry, and the
// wrong-result pricing variants selected by -DKB_ABL_* (tools/kbench/build.sh):
//   KB_ABL_NOLOAD=1   k_rows synthesises its inputs (no global loads)
//   KB_ABL_NOSTORE=1  k_rows folds its outputs into one conditional store (no stores)
//   KB_ABL_NOXCHG=1   no LDS exchanges
//   KB_ABL_L2LOAD=W   k_rows unit u reads unit u mod W (W units: L2- or Infinity-Cache-resident;
//                     with the tiled square split, W a multiple of 256 rows = whole polynomials)
//   KB_ABL_STROWS=W   k_rows unit u stores into unit W + u mod W (a window apart from the loads')
//   KB_ABL_L2CF=W     forward column pass: polynomial p reads polynomial p mod W (these are a, b)
//   KB_ABL_L2CI=W     inverse column pass: polynomial p reads polynomial p mod W
//   KB_ABL_STCF=W     forward column pass: polynomial p stores into polynomial W + p mod W
// Each is an NTTMUL_HOOK_* definition (the identity in the library, kernels_dev.hpp).
#if KB_ABL_NOLOAD
#define NTTMUL_HOOK_ROWS_INPUT(x, y, u, j)        \
  do {                                            \
    _Pragma("unroll") for (int k_ = 0; k_ < 16; k_++) { \
      x[k_] = (W)((j) * 16 + k_ + (u));           \
      y[k_] = (W)((j) * 7 + k_ * 3 + (u));        \
    }                                             \
  } while (0)
#endif
#if KB_ABL_NOSTORE
#define NTTMUL_HOOK_ROWS_OUTPUT(x, c, base, live)                       \
  do {                                                                  \
    W acc_ = 0;                                                         \
    _Pragma("unroll") for (int k_ = 0; k_ < 16; k_++) acc_ ^= x[k_];    \
    if (acc_ == (W)0x5A5A5A5A && (live)) (c)[base] = (TOut)acc_;        \
    return;                                                             \
  } while (0)
#endif
#if KB_ABL_NOXCHG
#define NTTMUL_HOOK_XCHG() return
#endif
#ifdef KB_ABL_L2LOAD
#define NTTMUL_HOOK_ROWS_LD(base, u, N, b0) ((base) - (size_t)((u) - (u) % (KB_ABL_L2LOAD)) * (N))
#endif
#ifdef KB_ABL_STROWS
#define NTTMUL_HOOK_ROWS_ST(base, u, N, b0) \
  ((base) - (size_t)((u) - (u) % (KB_ABL_STROWS) - (KB_ABL_STROWS)) * (N))
#endif
#if defined(KB_ABL_L2CF) && defined(KB_ABL_L2CI)
#define NTTMUL_HOOK_COLS_LD(base, p, sh, col, dir) \
  ((base) - ((size_t)((p) - (p) % ((dir) == 0 ? (KB_ABL_L2CF) : (KB_ABL_L2CI))) << (sh)))
#elif defined(KB_ABL_L2CF)
#define NTTMUL_HOOK_COLS_LD(base, p, sh, col, dir) \
  ((dir) == 0 ? (base) - ((size_t)((p) - (p) % (KB_ABL_L2CF)) << (sh)) : (base))
#elif defined(KB_ABL_L2CI)
#define NTTMUL_HOOK_COLS_LD(base, p, sh, col, dir) \
  ((dir) == 1 ? (base) - ((size_t)((p) - (p) % (KB_ABL_L2CI)) << (sh)) : (base))
#endif
#ifdef KB_ABL_STCF
#define NTTMUL_HOOK_COLS_ST(base, p, sh, col) \
  ((base) - ((size_t)((p) - (p) % (KB_ABL_STCF) - (KB_ABL_STCF)) << (sh)))
#endif
#include <hip/hip_runtime.h>
#include <type_traits>
// twiddle pairs of the transform stages (KB_SET 1's products):
//   KB_ABL_NOTW=1     synthesised from the table index in registers (no twiddle loads; one
//                     multiply per pair in their place; wrong results)
//   KB_TW_LDS=1       k_rows copies the forward and inverse pairs 0..511 (every pair a 4096-point
//                     product with 8-coefficient base blocks uses) into LDS once per workgroup and
//                     reads them there (exact for n <= 4096 with D = 3; other shapes not)
#if KB_ABL_NOTW
template <class T>
__device__ __forceinline__ T kb_notw(int idx) {
  using W = decltype(T::w);
  return T{(W)((uint32_t)idx * 0x9E3779B1u), (W)(uint32_t)idx};
}
#define NTTMUL_HOOK_TW(tw, idx, dir) kb_notw<std::remove_cv_t<std::remove_reference_t<decltype(*(tw))>>>(idx)
#endif
#if KB_TW_LDS
__shared__ uint2 kb_tws[2][512];
template <class T>
__device__ __forceinline__ void kb_stage_tw(const T *fw, const T *iw) {
  static_assert(sizeof(T) == 8, "u32 pairs");
  const uint4 *f4 = (const uint4 *)fw, *i4 = (const uint4 *)iw;
  uint4 *l4 = (uint4 *)&kb_tws[0][0];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {  // 2 x 512 pairs = 512 uint4
    l4[i] = f4[i];
    l4[256 + i] = i4[i];
  }
  __syncthreads();
}
template <class T>
__device__ __forceinline__ T kb_tw_lds(int idx, int dir) {
  const uint2 v = kb_tws[dir][idx & 511];
  return T{v.x, v.y};
}
#define NTTMUL_HOOK_ROWS_INPUT(x, y, u, j) kb_stage_tw(P.fw, P.iw)
#define NTTMUL_HOOK_TW(tw, idx, dir) \
  kb_tw_lds<std::remove_cv_t<std::remove_reference_t<decltype(*(tw))>>>(idx, dir)
#endif
// load order of a one-generation launch (C2: 4,096 one-wave products, 4 per SIMD, every wave's
// data lands late because the memory system interleaves all of their loads):
//   KB_PRIO_GEN=G     issue-priority variant only: unit u issues its loads at priority
//                     3 - min(3, u / G) (G = the units of one generation, 1,024 at C2), then
//                     returns to 3 once they are issued, so the first generation's loads queue
//                     ahead of the later ones' and its arithmetic starts while theirs stream in
//                     (exact)
#if KB_PRIO_GEN
__device__ __forceinline__ void kb_prio_gen(size_t u) {
  // (the priority ladder as one asm block with its own branches: compiler-visible branches here
  // moved the kernel's `live` select into VGPRs and wrapped every load in a waterfall loop)
  const uint32_t g = __builtin_amdgcn_readfirstlane((uint32_t)(u / (KB_PRIO_GEN)));
  asm volatile(
      "s_cmp_lt_u32 %0, 1\n\t"
      "s_cbranch_scc1 .Lkbp3_%=\n\t"
      "s_cmp_lt_u32 %0, 2\n\t"
      "s_cbranch_scc1 .Lkbp2_%=\n\t"
      "s_cmp_lt_u32 %0, 3\n\t"
      "s_cbranch_scc1 .Lkbp1_%=\n\t"
      "s_setprio 0\n\t"
      "s_branch .Lkbpe_%=\n"
      ".Lkbp1_%=:\n\t"
      "s_setprio 1\n\t"
      "s_branch .Lkbpe_%=\n"
      ".Lkbp2_%=:\n\t"
      "s_setprio 2\n\t"
      "s_branch .Lkbpe_%=\n"
      ".Lkbp3_%=:\n\t"
      "s_setprio 3\n"
      ".Lkbpe_%=:"
      :
      : "s"(g)
      : "scc");
}
#define NTTMUL_HOOK_PRIO0(u) kb_prio_gen(u)
#define NTTMUL_HOOK_ROWS_INPUT(x, y, u, j) __builtin_amdgcn_s_setprio(3)
#endif
// vector-memory instruction count of the coefficient streams (u32 products; wrong results):
//   KB_ABL_X4LOAD=1   a and b arrive by 16-byte loads (4 per polynomial per lane instead of 16
//                     dword loads), each lane's 16 consecutive-in-memory words landing in its
//                     registers unpermuted (the bytes of the product, a quarter of the instructions)
//   KB_ABL_X4STORE=1  c leaves by 16-byte stores the same way
typedef unsigned int kb_u4 __attribute__((ext_vector_type(4)));
#if KB_ABL_X4LOAD
#define NTTMUL_HOOK_ROWS_INPUT(x, y, u, j)                                                   \
  do {                                                                                      \
    const kb_u4 *pa_ = (const kb_u4 *)(a + (live ? u : 0) * N);                             \
    const kb_u4 *pb_ = (const kb_u4 *)(b + (live ? u : 0) * N);                             \
    _Pragma("unroll") for (int m_ = 0; m_ < 4; m_++) {                                      \
      const kb_u4 va_ = __builtin_nontemporal_load(pa_ + (j) + TP * m_);                    \
      const kb_u4 vb_ = __builtin_nontemporal_load(pb_ + (j) + TP * m_);                    \
      x[4 * m_] = va_.x; x[4 * m_ + 1] = va_.y; x[4 * m_ + 2] = va_.z; x[4 * m_ + 3] = va_.w; \
      y[4 * m_] = vb_.x; y[4 * m_ + 1] = vb_.y; y[4 * m_ + 2] = vb_.z; y[4 * m_ + 3] = vb_.w; \
    }                                                                                       \
  } while (0)
#endif
#if KB_ABL_X4STORE
#define NTTMUL_HOOK_ROWS_OUTPUT(x, c, base, live)                                  \
  do {                                                                             \
    if (live) {                                                                    \
      kb_u4 *pc_ = (kb_u4 *)((c) + u * N);                                         \
      _Pragma("unroll") for (int m_ = 0; m_ < 4; m_++) {                           \
        kb_u4 v_;                                                                  \
        v_.x = x[4 * m_]; v_.y = x[4 * m_ + 1]; v_.z = x[4 * m_ + 2]; v_.w = x[4 * m_ + 3]; \
        __builtin_nontemporal_store(v_, pc_ + j + TP * m_);                        \
      }                                                                            \
    }                                                                              \
    return;                                                                        \
  } while (0)
#endif
#ifndef KB_SET
#define KB_SET 1
#endif

#include "kernels_dev.hpp"
#include "kb.hpp"

namespace nttmul {
#if KB_PL
#include "kb_rows_pl.inc"
#endif

// C2 in-launch overlap experiments (each measured slower than k_rows at C2 and at
// n = 1024 x 262144, profiles/r3/c2/)
// Four independent one-wave products per 256-thread workgroup (n = 1024, u32 words): the k_rows
// product with exchanges ordered per wave (xsync<1>) instead of per workgroup, so a quarter of
// the workgroups to dispatch and no barrier coupling the four products.
template <class A, int LOGS>
__global__ __launch_bounds__(256) void k_rows_w4(KParams<A> P, const uint32_t *__restrict__ a,
                                                 const uint32_t *__restrict__ b,
                                                 uint32_t *__restrict__ c, size_t units) {
  using W = typename A::word;
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int N = Gr::N, NP = Gr::NP, G = Gr::G;
  static_assert(N / 16 == 64, "one wave per product");
  __shared__ W xch[4][NP];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), j = threadIdx.x & 63;
  const size_t u = (size_t)blockIdx.x * 4 + wv;
  if (u >= units) return;
  W *lx = xch[wv];
  constexpr int kAux = NTTMUL_CPOL < 0 ? 0 : NTTMUL_CPOL;
  constexpr int kAuxSt = NTTMUL_CPOL_ST < 0 ? 0 : NTTMUL_CPOL_ST;
  W x[16], y[16];
  const auto ra = span_rsrc(a + u * N, N), rb = span_rsrc(b + u * N, N);
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int off = (Gr::base(0, j) + Gr::off(0, k)) * 4;
    x[k] = (W)buf_ld32<kAux>(ra, off);
    y[k] = (W)buf_ld32<kAux>(rb, off);
  }
  constexpr int D = NTTMUL_BASE_D ? A::kBaseD : 0;
  TwPair<W> zw[16];
  fwd_all<A, LOGS, 0, 2, D, 1>(P.ar, x, y, lx, lx, P.fw, j, 0, 0, zw);
  base_mult<A, LOGS, D>(P.ar, x, y, zw, j);
  inv_all<A, LOGS, G - 1, true, D, 1>(P, x, y, lx, lx, P.iw, j, 0, 0);
  const auto rc = span_rsrc(c + u * N, N);
#pragma unroll
  for (int k = 0; k < 16; k++) {
    W v = x[k];
    if (!A::kInvCanonical) v = P.ar.canon(v);
    buf_st32<kAuxSt>(rc, (Gr::base(0, j) + Gr::off(0, k)) * 4, (uint32_t)v);
  }
}

// Pipelined one-wave products (n = 1024, u32 words): a 256-thread workgroup of four independent
// waves; each wave multiplies `per_wave` products in turn (units wave, wave + W, wave + 2W, ...,
// W = 4 gridDim.x) and issues the loads of its next product before it transforms the current
// one, so loads, arithmetic and stores of different products overlap inside one launch (a batch
// of 4096 one-wave products is otherwise a single generation: every wave loads, then computes,
// then stores, together).  The twiddles move to LDS once per workgroup (16 KiB), so a twiddle
// read never waits behind the prefetch in the in-order vector-memory counter; exchanges are
// ordered per wave (xsync<1>), so the four waves never wait for each other.
template <class A, int LOGS>
__global__ __launch_bounds__(256) void k_rows_pipe(KParams<A> P, const uint32_t *__restrict__ a,
                                                   const uint32_t *__restrict__ b,
                                                   uint32_t *__restrict__ c, size_t units) {
  using W = typename A::word;
  static_assert(sizeof(W) == 4, "u32 products");
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int N = Gr::N, NP = Gr::NP, G = Gr::G;
  static_assert(N / 16 == 64, "one wave per product");
  __shared__ TwPair<W> tws[2 * N];
  __shared__ W xch[4][NP];
  {  // both twiddle tables into LDS: 2 N pairs of 8 B, 16 B per thread per step
    const uint4 *fw4 = (const uint4 *)P.fw, *iw4 = (const uint4 *)P.iw;
    uint4 *t4 = (uint4 *)tws;
#pragma unroll
    for (int i = threadIdx.x; i < N / 2; i += 256) {
      t4[i] = fw4[i];
      t4[N / 2 + i] = iw4[i];
    }
  }
  __syncthreads();
  // (readfirstlane: the wave index is wave-uniform, so the buffer descriptors are scalar)
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), j = threadIdx.x & 63;
  const size_t stride = (size_t)gridDim.x * 4;
  size_t u = (size_t)blockIdx.x * 4 + wv;
  if (u >= units) return;
  W *lx = xch[wv];
  const TwPair<W> *fw = tws, *iw = tws + N;
  constexpr int kAux = NTTMUL_CPOL < 0 ? 0 : NTTMUL_CPOL;
  constexpr int kAuxSt = NTTMUL_CPOL_ST < 0 ? 0 : NTTMUL_CPOL_ST;
  W x[16], y[16], nx[16], ny[16];
  {
    const auto ra = span_rsrc(a + u * N, N), rb = span_rsrc(b + u * N, N);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int off = (Gr::base(0, j) + Gr::off(0, k)) * 4;
      x[k] = (W)buf_ld32<kAux>(ra, off);
      y[k] = (W)buf_ld32<kAux>(rb, off);
    }
  }
  constexpr int D = NTTMUL_BASE_D ? A::kBaseD : 0;
  for (;;) {
    const size_t un = u + stride;
    const bool more = un < units;  // wave-uniform
    {  // unconditional (the last product reloads itself), pinned ahead of the transforms
      const size_t ul = more ? un : u;
      const auto ra = span_rsrc(a + ul * N, N), rb = span_rsrc(b + ul * N, N);
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const int off = (Gr::base(0, j) + Gr::off(0, k)) * 4;
        nx[k] = (W)buf_ld32<kAux>(ra, off);
        ny[k] = (W)buf_ld32<kAux>(rb, off);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    TwPair<W> zw[16];
    fwd_all<A, LOGS, 0, 2, D, 1>(P.ar, x, y, lx, lx, fw, j, 0, 0, zw);
    base_mult<A, LOGS, D>(P.ar, x, y, zw, j);
    inv_all<A, LOGS, G - 1, true, D, 1>(P, x, y, lx, lx, iw, j, 0, 0);
    {
      const auto rc = span_rsrc(c + u * N, N);
#pragma unroll
      for (int k = 0; k < 16; k++) {
        W v = x[k];
        if (!A::kInvCanonical) v = P.ar.canon(v);
        buf_st32<kAuxSt>(rc, (Gr::base(0, j) + Gr::off(0, k)) * 4, (uint32_t)v);
      }
    }
    if (!more) break;
    u = un;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      x[k] = nx[k];
      y[k] = ny[k];
    }
  }
}

// Two waves per product (n = 1024, u32 words): wave 0 transforms a, wave 1 transforms b at the
// same time, wave 1 hands its transformed b to wave 0 through LDS (register k of lane j at word
// 64 k + j: the same element in both waves) and exits; wave 0 multiplies, runs the inverse and
// stores.  Each wave holds one polynomial, so twice the waves fit per SIMD, and the longest
// per-wave chain is two thirds of a product's work instead of all of it.
template <class A, int LOGS>
__global__ __launch_bounds__(128) void k_rows_ab(KParams<A> P, const uint32_t *__restrict__ a,
                                                 const uint32_t *__restrict__ b,
                                                 uint32_t *__restrict__ c, size_t units) {
  using W = typename A::word;
  static_assert(sizeof(W) == 4, "u32 products");
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int N = Gr::N, NP = Gr::NP, G = Gr::G;
  static_assert(N / 16 == 64 && NP >= N, "one wave per polynomial");
  __shared__ W xch[2][NP];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), j = threadIdx.x & 63;
  const size_t u = blockIdx.x;
  if (u >= units) return;  // block-uniform
  W *lx = xch[wv];
  constexpr int kAux = NTTMUL_CPOL < 0 ? 0 : NTTMUL_CPOL;
  constexpr int kAuxSt = NTTMUL_CPOL_ST < 0 ? 0 : NTTMUL_CPOL_ST;
  W x[16], y[16];
  {
    const auto r = span_rsrc((wv ? b : a) + u * N, N);
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = (W)buf_ld32<kAux>(r, (Gr::base(0, j) + Gr::off(0, k)) * 4);
  }
  constexpr int D = NTTMUL_BASE_D ? A::kBaseD : 0;
  TwPair<W> zw[16];
  fwd_all<A, LOGS, 0, 1, D, 1>(P.ar, x, y, lx, lx, P.fw, j, 0, 0, zw);
  if (wv) {
    W *t = xch[1];
    xsync<1>();  // wave 1's last exchange reads are done before the region is overwritten
#pragma unroll
    for (int k = 0; k < 16; k++) t[k * 64 + j] = x[k];
  }
  __syncthreads();
  if (wv) return;
#pragma unroll
  for (int k = 0; k < 16; k++) y[k] = xch[1][k * 64 + j];
  base_mult<A, LOGS, D>(P.ar, x, y, zw, j);
  inv_all<A, LOGS, G - 1, true, D, 1>(P, x, y, lx, lx, P.iw, j, 0, 0);
  const auto rc = span_rsrc(c + u * N, N);
#pragma unroll
  for (int k = 0; k < 16; k++) {
    W v = x[k];
    if (!A::kInvCanonical) v = P.ar.canon(v);
    buf_st32<kAuxSt>(rc, (Gr::base(0, j) + Gr::off(0, k)) * 4, (uint32_t)v);
  }
}


// ---------------------------------------------------------------------------------------------
// Persistent, phase-pipelined multi-pass product (n = 2^L1 * 4096 > 4096): measured slower than
// the three launches (profiles/r3/c5_persist/), so the library does not carry it
// (no product path of libnttmul.so can return after a given-up dependency wait)
// ---------------------------------------------------------------------------------------------
// The three passes of multipass_l1 (k_cols_fwd -> k_rows<..., 12, L1> -> k_cols_inv) as tasks of
// ONE launch: a grid of resident workgroups pulls tickets from a device-side counter.  Per
// polynomial p there are kMpCols column-forward tasks CF(p, s) (256 columns each, all 2^L1
// elements of each column), 2^L1 row tasks R(p, r) and kMpCols column-inverse tasks CI(p, s).
// R(p, .) needs every CF(p, .), CI(p, .) every R(p, .).  Ticket t belongs to step k = t / T with
// T = 2 kMpCols + 2^L1 tasks: first the CI tasks of polynomial k - 2 lag, then the R tasks of
// k - lag, then the CF tasks of k.  A task's dependencies therefore hold smaller tickets, which
// were handed to running workgroups earlier: the smallest unfinished ticket can always run, so
// the schedule cannot deadlock, and with lag steps between producer and consumer the wait is
// normally over before the consumer starts.  No relaunch, no grid-wide ramp and drain between
// passes; the memory-bound column tasks of younger polynomials run beside the VALU-bound row tasks
// of older ones on the same CUs, and an intermediate is read back about 2 lag steps (~2 lag x
// 1.5 MiB for C5) after it was written, while it is still in the 256 MiB Infinity Cache.
//
// Hand-off (MI355X_MICROARCH.md §inter-workgroup visibility, table row 1): every intermediate is
// stored with sc1 stores (write-through; a cross-XCD reader then cannot see a stale copy in its
// own L2 once the data reached memory) and read with sc1 loads (L1 bypassed); each storing wave
// waits vmcnt(0), the workgroup barriers, and one lane adds 1 (agent scope) to the polynomial's
// counter; a consumer's lane 0 polls that counter with sc1 loads, then the workgroup barriers.
// Every scratch word is written once and read once per launch (no address reuse inside a
// launch).  A poll that has not seen its count after 2^20 polls (tens of ms to ~1 s, far beyond
// any wait of a correct schedule) records a fault flag and gives up, so a bug ends the launch
// instead of hanging the GPU.
constexpr int kMpCols = 16;  // column tasks per polynomial: 4096 columns / 256 threads
struct MpSync {
  unsigned *head;            // ticket counter (zeroed before the launch)
  unsigned *cnt;             // [2][batch]: finished CF / R tasks per polynomial (zeroed)
  unsigned *fault;           // set when a poll gave up
  unsigned lag;              // steps between a polynomial's CF, R and CI tasks
  unsigned long long *stats; // tools/kbench NTTMUL_MP_STATS builds: per task type (CI, R, CF)
                             // [0..2] busy ticks, [3..5] wait ticks, [6..8] tasks (100 MHz clock)
};
#ifndef NTTMUL_MP_STATS
#define NTTMUL_MP_STATS 0
#endif
// sc1 hand-off policy of the intermediates (2 = sc1 loads and stores; kbench A/B only: 0 plain)
#ifndef NTTMUL_MP_POL
#define NTTMUL_MP_POL 2
#endif

template <int POL, class T>
__device__ __forceinline__ T ld_pol(const T *p) {
  if constexpr (POL == 2) return __hip_atomic_load((T *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else if constexpr (POL == 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int POL, class T>
__device__ __forceinline__ void st_pol(T *p, T v) {
  if constexpr (POL == 2) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else if constexpr (POL == 1) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// the storing workgroup's release: every wave's stores complete, then one lane counts the task
__device__ __forceinline__ void mp_publish(unsigned *cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
// the consuming workgroup's wait for `need` finished producer tasks
__device__ __forceinline__ void mp_wait(const MpSync &S, const unsigned *cnt, unsigned need) {
  if (threadIdx.x == 0) {
    unsigned polls = 0;
    while (__hip_atomic_load((unsigned *)cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < need) {
      __builtin_amdgcn_s_sleep(2);
      if (++polls == (1u << 20)) {  // >= 60 ms of polling: far beyond any correct wait
        __hip_atomic_store(S.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  // the producers' stores, made visible by their release, before any lane of this workgroup loads
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

__device__ __forceinline__ void mp_stat(const MpSync &S, int kind, unsigned long long t0,
                                        unsigned long long t1) {
  if (NTTMUL_MP_STATS && threadIdx.x == 0) {
    const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    atomicAdd(S.stats + kind, t2 - t1);
    atomicAdd(S.stats + 3 + kind, t1 - t0);
    atomicAdd(S.stats + 6 + kind, 1ull);
  }
}

template <class A, class IO, int L1>
__global__ __launch_bounds__(256) void k_mp_persist(KParams<A> P, const IO *__restrict__ a,
                                                    const IO *__restrict__ b, IO *__restrict__ c,
                                                    typename A::word *__restrict__ ta,
                                                    typename A::word *__restrict__ tb,
                                                    typename A::word *__restrict__ tc,
                                                    unsigned batch, MpSync S) {
  using W = typename A::word;
  constexpr int LOGS = 12, NR = 1 << L1, M = 1 << L1;
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int N = Gr::N, G = Gr::G, NP = Gr::NP;
  constexpr unsigned T = 2 * kMpCols + NR;
  constexpr size_t kPoly = (size_t)N << L1;   // words per polynomial
  __shared__ W lds[NP];
  __shared__ unsigned s_ticket;
  const int j = threadIdx.x;
  const unsigned total = (batch + 2 * S.lag) * T;
  if (j == 0) s_ticket = __hip_atomic_fetch_add(S.head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  unsigned t = s_ticket;
  while (t < total) {
    __syncthreads();  // every lane has read s_ticket
    if (j == 0) s_ticket = __hip_atomic_fetch_add(S.head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned k = t / T, r = t % T;
    if (r < kMpCols) {
      // CI(p, r): inverse column stages L1-1 .. 0 with F folded into stage 0, canonical output
      if (k >= 2 * S.lag && k - 2 * S.lag < batch) {
        const size_t p = k - 2 * S.lag;
        const unsigned long long t0 = NTTMUL_MP_STATS ? __builtin_amdgcn_s_memrealtime() : 0;
        mp_wait(S, S.cnt + batch + p, NR);
        const unsigned long long t1 = NTTMUL_MP_STATS ? __builtin_amdgcn_s_memrealtime() : 0;
        const size_t base = p * kPoly + (size_t)r * 256 + j;
        W x[M];
#pragma clang loop unroll(full)
        for (int m = 0; m < M; m++) x[m] = ld_pol<NTTMUL_MP_POL>(tc + base + ((size_t)m << LOGS));
#pragma clang loop unroll(full)
        for (int st = L1 - 1; st >= 0; st--) {
          const int dist = M >> (st + 1);
#pragma clang loop unroll(full)
          for (int m = 0; m < M; m++) {
            if (m & dist) continue;
            if (st == 0) {
              P.ar.gs_scaled(x[m], x[m + dist], P.f, P.fs, P.wf, P.wfs);
            } else {
              const TwPair<W> tw = P.iw[(1 << st) + (m >> (L1 - st))];
              P.ar.gs(x[m], x[m + dist], tw.w, tw.ws);
            }
          }
        }
#pragma clang loop unroll(full)
        for (int m = 0; m < M; m++)
          st_pol<1>(c + base + ((size_t)m << LOGS), (IO)(A::kInvCanonical ? x[m] : P.ar.canon(x[m])));
        if (NTTMUL_MP_STATS) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __syncthreads();
          mp_stat(S, 0, t0, t1);
        }
      }
    } else if (r < kMpCols + NR) {
      // R(p, row): row stages L1 .. L1 + 11, base multiplication, inverse row stages; lazy out
      if (k >= S.lag && k - S.lag < batch) {
        const size_t p = k - S.lag;
        const int row = (int)(r - kMpCols);
        const unsigned long long t0 = NTTMUL_MP_STATS ? __builtin_amdgcn_s_memrealtime() : 0;
        mp_wait(S, S.cnt + p, kMpCols);
        const unsigned long long t1 = NTTMUL_MP_STATS ? __builtin_amdgcn_s_memrealtime() : 0;
        const size_t base = p * kPoly + ((size_t)row << LOGS) + Gr::base(0, j);
        W x[16], y[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
          x[q] = ld_pol<NTTMUL_MP_POL>(ta + base + Gr::off(0, q));
          y[q] = ld_pol<NTTMUL_MP_POL>(tb + base + Gr::off(0, q));
        }
        constexpr int D = NTTMUL_BASE_D ? A::kBaseD : 0;
        TwPair<W> zw[16];
        fwd_all<A, LOGS, 0, 2, D>(P.ar, x, y, lds, lds, P.fw, j, row, L1, zw);
        base_mult<A, LOGS, D>(P.ar, x, y, zw, j);
        inv_all<A, LOGS, G - 1, false, D>(P, x, y, lds, lds, P.iw, j, row, L1);
#pragma unroll
        for (int q = 0; q < 16; q++) st_pol<NTTMUL_MP_POL>(tc + base + Gr::off(0, q), x[q]);
        mp_publish(S.cnt + batch + p);
        mp_stat(S, 1, t0, t1);
      }
    } else {
      // CF(p, s): forward column stages 0 .. L1-1 of a and b
      if (k < batch) {
        const size_t p = k;
        const unsigned long long t0 = NTTMUL_MP_STATS ? __builtin_amdgcn_s_memrealtime() : 0;
        const size_t base = p * kPoly + (size_t)(r - kMpCols - NR) * 256 + j;
        W x[M], y[M];
#pragma clang loop unroll(full)
        for (int m = 0; m < M; m++) {
          x[m] = (W)ld_pol<NTTMUL_NT_COLS>(a + base + ((size_t)m << LOGS));
          y[m] = (W)ld_pol<NTTMUL_NT_COLS>(b + base + ((size_t)m << LOGS));
        }
#pragma clang loop unroll(full)
        for (int st = 0; st < L1; st++) {
          const int dist = M >> (st + 1);
#pragma clang loop unroll(full)
          for (int m = 0; m < M; m++) {
            if (m & dist) continue;
            const TwPair<W> tw = P.fw[(1 << st) + (m >> (L1 - st))];
            P.ar.ct(x[m], x[m + dist], tw.w, tw.ws);
            P.ar.ct(y[m], y[m + dist], tw.w, tw.ws);
          }
        }
#pragma clang loop unroll(full)
        for (int m = 0; m < M; m++) {
          st_pol<NTTMUL_MP_POL>(ta + base + ((size_t)m << LOGS), x[m]);
          st_pol<NTTMUL_MP_POL>(tb + base + ((size_t)m << LOGS), y[m]);
        }
        mp_publish(S.cnt + p);
        mp_stat(S, 2, t0, t0);
      }
    }
    __syncthreads();  // s_ticket written by lane 0 above
    t = s_ticket;
  }
}


}  // namespace nttmul

namespace kb {
using namespace nttmul;

// Pipelined n = 1024 products (k_rows_pipe): pipe_per_wave products per wave (the grid covers the
// batch with ceil(batch / (4 per_wave)) four-wave workgroups).
template <class A>
static hipError_t launch_pipe(const KParams<A> &P, const void *a, const void *b, void *c,
                              size_t units, int per_wave, hipStream_t s) {
  const size_t per_block = 4 * (size_t)per_wave;
  const size_t blocks = (units + per_block - 1) / per_block;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((k_rows_pipe<A, 10>), dim3((unsigned)blocks), dim3(256), 0, s, P,
                     (const uint32_t *)a, (const uint32_t *)b, (uint32_t *)c, units);
  return hipGetLastError();
}

template <class A>
static hipError_t fused(const LaunchTables &T, const Conf &C, const void *a, const void *b,
                        void *c, size_t batch, hipStream_t s) {
  const KParams<A> P = product_params<A>(T);
  if constexpr (std::is_same<A, Arith32P>::value) {
    if (T.logn == 10 && C.pipe_per_wave > 0)
      return launch_pipe<A>(P, a, b, c, batch, C.pipe_per_wave, s);
    if (T.logn == 10 && C.pipe_per_wave == -2) {  // k_rows_ab
      if (batch == 0) return hipSuccess;
      hipLaunchKernelGGL((k_rows_ab<A, 10>), dim3((unsigned)batch), dim3(128), 0, s, P,
                         (const uint32_t *)a, (const uint32_t *)b, (uint32_t *)c, batch);
      return hipGetLastError();
    }
    if (T.logn == 10 && C.pipe_per_wave == -1) {  // k_rows_w4
      const size_t blocks = (batch + 3) / 4;
      if (blocks == 0) return hipSuccess;
      hipLaunchKernelGGL((k_rows_w4<A, 10>), dim3((unsigned)blocks), dim3(256), 0, s, P,
                         (const uint32_t *)a, (const uint32_t *)b, (uint32_t *)c, batch);
      return hipGetLastError();
    }
  }
#if KB_PL
  // KB_PL: the n = 1024 product through k_rows_pl (tools/kbench/gen_rows_pl.py: the same kernel,
  // arguments a, b, c, units first so -amdgpu-kernarg-preload-count can preload them)
  if constexpr (IsPlantard<A>::value) {
    if (T.logn == 10) {
      constexpr int NT = rows_threads(10), PB = NT / 64;
      const size_t blocks = (batch + PB - 1) / PB;
      if (blocks == 0) return hipSuccess;
      const bool prio = rows_prio(blocks * (NT / 64));
      if (prio)
        hipLaunchKernelGGL((k_rows_pl<A, uint32_t, uint32_t, 10, 0, true>), dim3((unsigned)blocks),
                           dim3(NT), 0, s, (const uint32_t *)a, (const uint32_t *)b,
                           (uint32_t *)c, batch, P);
      else
        hipLaunchKernelGGL((k_rows_pl<A, uint32_t, uint32_t, 10, 0>), dim3((unsigned)blocks),
                           dim3(NT), 0, s, (const uint32_t *)a, (const uint32_t *)b,
                           (uint32_t *)c, batch, P);
      return hipGetLastError();
    }
  }
#endif
  switch (T.logn) {
    case 8: return launch_rows<A, uint32_t, uint32_t, 8, 0>(P, a, b, c, batch, s);
    case 9: return launch_rows<A, uint32_t, uint32_t, 9, 0>(P, a, b, c, batch, s);
    case 10: return launch_rows<A, uint32_t, uint32_t, 10, 0>(P, a, b, c, batch, s);
    case 11: return launch_rows<A, uint32_t, uint32_t, 11, 0>(P, a, b, c, batch, s);
    case 12: return launch_rows<A, uint32_t, uint32_t, 12, 0>(P, a, b, c, batch, s);
    default: return hipErrorInvalidValue;
  }
}

// The library's three-launch multi-pass product (kernels.hip multipass_l1), one pass at a time
// when C.mp_phase >= 0, the row pass with C.rows_lds_extra bytes of dynamic LDS
template <class A, class IO, int L1, int LOGS = 12>
static hipError_t multipass_l1(const LaunchTables &T, const Conf &C, const void *a, const void *b,
                               void *c, size_t batch, void *ta, void *tb, void *tc, hipStream_t s) {
  using W = typename A::word;
  const KParams<A> P = product_params<A>(T);
  const unsigned cblocks = (unsigned)(((batch << LOGS) + 255) / 256);
  hipError_t e = hipSuccess;
  if (C.mp_phase < 0 || C.mp_phase == 0) {
    hipLaunchKernelGGL((k_cols_fwd<A, IO, L1>), dim3(cblocks), dim3(256), 0, s, P, (const IO *)a,
                       (const IO *)b, (W *)ta, (W *)tb, batch, LOGS);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (C.mp_phase < 0 || C.mp_phase == 1) {
    constexpr size_t PB = 256 / ((1 << LOGS) / 16);
    const size_t units = batch << L1, blocks = (units + PB - 1) / PB;
    hipLaunchKernelGGL((k_rows<A, W, W, LOGS, L1>), dim3((unsigned)blocks), dim3(256),
                       (unsigned)C.rows_lds_extra, s, P, (const W *)ta, (const W *)tb, (W *)tc,
                       units);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (C.mp_phase < 0 || C.mp_phase == 2) {
    hipLaunchKernelGGL((k_cols_inv<A, IO, L1>), dim3(cblocks), dim3(256), 0, s, P,
                       (const W *)tc, (IO *)c, batch, LOGS);
    e = hipGetLastError();
  }
  return e;
}

// The library's square split (kernels.hip multipass_sq, NTTMUL_C5_SQ): k_cols8 forward, the row
// pass of 256-coefficient rows, k_cols8 inverse; phases and row-pass LDS as multipass_l1
template <class A, class IO>
static hipError_t multipass_sq(const LaunchTables &T, const Conf &C, const void *a, const void *b,
                               void *c, size_t batch, void *ta, void *tb, void *tc, hipStream_t s) {
  using W = typename A::word;
  const KParams<A> P = product_params<A>(T);
  const size_t groups = batch * 16;
  hipError_t e = hipSuccess;
  if (C.mp_phase < 0 || C.mp_phase == 0) {
    hipLaunchKernelGGL((k_cols8<A, IO, W, 0>), dim3((unsigned)groups), dim3(256), 0, s, P,
                       (const IO *)a, (const IO *)b, (W *)ta, (W *)tb, groups);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (C.mp_phase < 0 || C.mp_phase == 1) {
    const size_t units = batch << 8, blocks = (units + 15) / 16;
    hipLaunchKernelGGL((k_rows<A, W, W, 8, 8>), dim3((unsigned)blocks), dim3(256),
                       (unsigned)C.rows_lds_extra, s, P, (const W *)ta, (const W *)tb, (W *)tc,
                       units);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (C.mp_phase < 0 || C.mp_phase == 2) {
    hipLaunchKernelGGL((k_cols8<A, W, IO, 1>), dim3((unsigned)groups), dim3(256), 0, s, P,
                       (const W *)tc, (const W *)nullptr, (IO *)c, (IO *)nullptr, groups);
    e = hipGetLastError();
  }
  return e;
}

// The same product in one persistent launch (k_mp_persist).  scr[3]: the ticket / counter words,
// mp_sync_bytes(batch), zeroed here on the stream before the launch.
template <class A, class IO, int L1>
static hipError_t multipass_persist(const LaunchTables &T, const Conf &C, const void *a,
                                    const void *b, void *c, size_t batch, void **scr,
                                    hipStream_t s) {
  using W = typename A::word;
  if (batch == 0) return hipSuccess;
  if (batch > 0x7FFFFFFFull / (2 * kMpCols + (1 << L1))) return hipErrorInvalidValue;
  static const int per_cu = [] {  // resident workgroups per CU (occupancy of this instantiation)
    int k = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &k, reinterpret_cast<const void *>(&k_mp_persist<A, IO, L1>), 256, 0);
    return e != hipSuccess || k < 1 ? 1 : k;
  }();
  const KParams<A> P = product_params<A>(T);
  unsigned *sw = (unsigned *)scr[3];
  hipError_t e = hipMemsetAsync(sw, 0, mp_sync_bytes(batch), s);
  if (e != hipSuccess) return e;
  MpSync S;
  S.head = sw;
  S.fault = sw + 1;
  S.cnt = sw + 2;
  S.lag = (unsigned)(C.mp_lag < 4096 ? C.mp_lag : 4096);  // (batch + 2 lag) T stays far below 2^32
  if ((batch + 2 * (size_t)S.lag) * (32 + (1u << L1)) >= (1ull << 31)) return hipErrorInvalidValue;
  S.stats = (unsigned long long *)C.mp_stats;
  const unsigned grid = (unsigned)(per_cu * (T.cus > 0 ? T.cus : 256));
  hipLaunchKernelGGL((k_mp_persist<A, IO, L1>), dim3(grid), dim3(256), 0, s, P, (const IO *)a,
                     (const IO *)b, (IO *)c, (W *)scr[0], (W *)scr[1], (W *)scr[2],
                     (unsigned)batch, S);
  return hipGetLastError();
}

static hipError_t launch_(const LaunchTables &T, const Conf &C, const void *a, const void *b,
                          void *c, size_t batch, int io_bits, void **scr, hipStream_t s);
// the library's launch_polymul rule for the issue-priority variant (kernels_dev.hpp rows_prio):
// one-generation launches of the Plantard kernels take it (C2), unless T.prio says otherwise
hipError_t launch(const LaunchTables &T, const Conf &C, const void *a, const void *b, void *c,
                  size_t batch, int io_bits, void **scr, hipStream_t s) {
  const int prev = tl_prio_cus, prev_mode = tl_prio_mode;
  tl_prio_cus = T.prio_ok ? T.cus : 0;
  tl_prio_mode = T.prio;
  const hipError_t e = launch_(T, C, a, b, c, batch, io_bits, scr, s);
  tl_prio_cus = prev;
  tl_prio_mode = prev_mode;
  return e;
}
static hipError_t launch_(const LaunchTables &T, const Conf &C, const void *a, const void *b,
                          void *c, size_t batch, int io_bits, void **scr, hipStream_t s) {
#if KB_SET == 2  // C5: 64-bit words, n = 65536
  if (T.word_bits != 64 || T.logn != 16 || io_bits != 64) return hipErrorNotSupported;
  if (C.mp_lag > 0 && scr[3])
    return multipass_persist<Arith64, uint64_t, 4>(T, C, a, b, c, batch, scr, s);
  if (NTTMUL_C5_SQ)
    return multipass_sq<Arith64, uint64_t>(T, C, a, b, c, batch, scr[0], scr[1], scr[2], s);
  return multipass_l1<Arith64, uint64_t, 4>(T, C, a, b, c, batch, scr[0], scr[1], scr[2], s);
#else  // u32 words, q < 2^31, n <= 4096
  if (T.word_bits != 32 || T.q >= (1ull << 31) || T.logn > 12 || io_bits != 32)
    return hipErrorNotSupported;
  switch (a32_kind(T.q)) {
    case A32Kind::Harvey: return fused<Arith32H>(T, C, a, b, c, batch, s);
    case A32Kind::Plantard:
      if (T.logn == 12 && p3_fold_ok(T.q))
        return launch_rows<Arith32P3, uint32_t, uint32_t, 12, 0>(product_params<Arith32P3>(T), a,
                                                                 b, c, batch, s);
      return fused<Arith32P>(T, C, a, b, c, batch, s);
    default: return fused<Arith32>(T, C, a, b, c, batch, s);
  }
#endif
}

hipError_t fill(void *a, void *b, uint32_t logn, uint64_t q, uint64_t seed, size_t count,
                int io_bits, hipStream_t s) {
  const size_t total = count << logn;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  if (!total) return hipSuccess;
  if (io_bits == 32)
    hipLaunchKernelGGL(k_fill<uint32_t>, dim3(blocks), dim3(256), 0, s, (uint32_t *)a,
                       (uint32_t *)b, logn, q, seed, (uint64_t)0, total);
  else
    hipLaunchKernelGGL(k_fill<uint64_t>, dim3(blocks), dim3(256), 0, s, (uint64_t *)a,
                       (uint64_t *)b, logn, q, seed, (uint64_t)0, total);
  return hipGetLastError();
}

const char *set_name() { return KB_SET == 2 ? "C5 (u64, n = 65536)" : "u32, q < 2^31, n <= 4096"; }

}  // namespace kb
