// kernels_dev.hpp — gfx950 kernels of the negacyclic polynomial product c = a * b mod (x^n + 1, q)
// (device code; the library's launchers are in kernels.hip, tools/kbench's in its own sources).
#pragma once
//
// Algorithm (reference = NTT_Software/NTT_Software_Evaluations/NTT-256/NTT/ntt.C):
//   forward  : mulntt_ct_std2rev (ntt.C:342-371) — psi-merged Cooley-Tukey, standard order in,
//              bit-reversed out, twiddle p[t+j] = psi^(n/2t) omega^((n/2t) bitrev(j))
//   pointwise: mul_array (ntt.C:131-137) in the bit-reversed domain (order-agnostic)
//   inverse  : nttmul_gs_rev2std (ntt.C:428-451) — psi^-1-merged Gentleman-Sande, bit-reversed
//              in, standard out; the n^-1 of ntt256.C:12 is folded into the last stage
// Every butterfly of forward-stage index st (t = 2^st, distance d = n >> (st+1)) acting on lower
// element e uses twiddle index 2^st + (e >> (logn - st)) in both directions (the inverse runs the
// same stages in reverse order).  No bit-reversal permutation is ever materialised.
//
// Kernel shapes
//   k_rows   : fused per polynomial (n <= 4096): 256-thread block, 16 coefficients per thread,
//              stages in register groups of <= 4 (radix-16), LDS transposes between groups,
//              a and b transformed together (shared twiddle loads), pointwise, inverse, store.
//              For n > 4096 the same kernel is the "row" pass of a two-level decomposition
//              n = 2^L1 * 2^LOGS: rows are contiguous 2^LOGS-blocks whose stages are the last LOGS.
//   k_cols_* : the first L1 <= 4 stages for n > 4096 (column pass), one column per thread in
//              registers, lanes on consecutive columns (coalesced), no LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <string>
#include <type_traits>

#include "launch.hpp"
#include "modarith.hpp"

// LDS regions per polynomial pair for 32-bit words (2: a and b exchanged together; 1: in turn,
// half the LDS).  One region: 17 KiB per n = 4096 block, 7 blocks (VGPR-limited) instead of 4 per
// CU; with the Plantard kernel -2 % at C3, -1 % at n = 1024 x 262144 and n = 65536, C2 unchanged
// (profiles/r2/plantard/ab1.txt).  64-bit words always use one region (C5 -6 %, tools/c5_ab.sh)
#ifndef NTTMUL_LDS_REGIONS
#define NTTMUL_LDS_REGIONS 1
#endif
// a, b, c streams of the one-product-per-block u32 products (n = 4096, 1024) as buffer loads /
// stores on a block-uniform descriptor with cache-policy bits aux = NTTMUL_CPOL (1 sc0, 2 nt,
// 16 sc1; -1: global loads as below).  C3 kbench A/B (profiles/r2/cpol_ab.txt, identical
// checksums): nt -1.2 % against the global nt loads (the 32-bit voffset form drops the 64-bit
// address adds: 1,940 VALU per wave instead of 1,951); nt with sc0 / sc1 the same as nt alone;
// plain (0) +0.3 %, sc1 alone +0.1 %
#ifndef NTTMUL_CPOL
#define NTTMUL_CPOL 2
#endif
#ifndef NTTMUL_CPOL_ST
#define NTTMUL_CPOL_ST NTTMUL_CPOL
#endif
// non-temporal loads/stores of the coefficient streams in k_rows
#ifndef NTTMUL_NT
#define NTTMUL_NT 1
#endif
// n = 1024: a's loads first and a's forward transform before b's (k_rows kSplitAB)
#ifndef NTTMUL_SPLIT_AB
#define NTTMUL_SPLIT_AB 0
#endif
// NTTMUL_A32H / NTTMUL_A32_PLANTARD (which 32-bit class takes which q): arith_select.hpp
// incomplete transforms in the product kernel: the last D = A::kBaseD stages become base
// multiplications of 2^D-coefficient blocks (0: full transforms + pointwise Montgomery product)
#ifndef NTTMUL_BASE_D
#define NTTMUL_BASE_D 1
#endif
// skip the reduction of X in the first forward stage (input canonical by contract)
#ifndef NTTMUL_FIRST_XC
#define NTTMUL_FIRST_XC 1
#endif
// __launch_bounds__ minimum waves per SIMD for k_rows (1 = no constraint)
#ifndef NTTMUL_MIN_WAVES
#define NTTMUL_MIN_WAVES 1
#endif
// conflict-free LDS padding for the group 0 <-> 1 exchanges (Groups::padx; 0 = e + (e >> 4))
#ifndef NTTMUL_PAD0
#define NTTMUL_PAD0 1
#endif
// two-term pads at n = 512 / 1024 (Groups::PS2)
#ifndef NTTMUL_PAD2
#define NTTMUL_PAD2 1
#endif
// NTTMUL_SPLIT16 (column stages of the n = 65536 multi-pass product): arith_select.hpp
// Instrumentation points, the identity here.  tools/kbench/kb_hooks.hpp defines them before it
// includes this header, to build wrong-result pricing variants of these same kernels (loads or
// stores redirected into an L2- or Infinity-Cache-sized window, inputs synthesised instead of
// loaded, stores or LDS exchanges dropped).  csrc/kernels.hip, the library's
// translation unit, stops with #error if any of them is defined before it includes this file.
//   NTTMUL_HOOK_ROWS_LD(base, u, N, b0)     k_rows: word offset its loads start from
//   NTTMUL_HOOK_ROWS_ST(base, u, N, b0)     k_rows (global-store path): word offset of its stores
//   NTTMUL_HOOK_ROWS_INPUT(x, y, u, j)      k_rows: statement after the loads (may overwrite x, y)
//   NTTMUL_HOOK_ROWS_OUTPUT(x, c, base, live) k_rows: statement before the stores (may return)
//   NTTMUL_HOOK_XCHG()                      exchange: statement before the LDS round trip
//   NTTMUL_HOOK_PRIO0(u)                    k_rows issue-priority variant: the statement that
//                                           sets the wave's priority before its loads
//   NTTMUL_HOOK_TW(tw, idx, dir)            transform stages (untyped twiddle tables; dir 0
//                                           forward, 1 inverse): the pair tw[idx]
//   NTTMUL_HOOK_COLS_LD(base, p, sh, col, dir) column passes (dir 0 forward, 1 inverse): word
//                                           offset their loads start from
//   NTTMUL_HOOK_COLS_ST(base, p, sh, col)   column passes: word offset of the intermediates' stores
#if defined(NTTMUL_HOOK_ROWS_LD) || defined(NTTMUL_HOOK_ROWS_ST)
#define NTTMUL_ROWS_HOOKED 1  // (kbench pricing builds: the row pass keeps global addressing)
#else
#define NTTMUL_ROWS_HOOKED 0
#endif
#ifndef NTTMUL_HOOK_ROWS_LD
#define NTTMUL_HOOK_ROWS_LD(base, u, N, b0) (base)
#endif
#ifndef NTTMUL_HOOK_ROWS_ST
#define NTTMUL_HOOK_ROWS_ST(base, u, N, b0) (base)
#endif
#ifndef NTTMUL_HOOK_ROWS_INPUT
#define NTTMUL_HOOK_ROWS_INPUT(x, y, u, j) do { } while (0)
#endif
#ifndef NTTMUL_HOOK_ROWS_OUTPUT
#define NTTMUL_HOOK_ROWS_OUTPUT(x, c, base, live) do { } while (0)
#endif
#ifndef NTTMUL_HOOK_PRIO0
#define NTTMUL_HOOK_PRIO0(u) __builtin_amdgcn_s_setprio(3)
#endif
#ifndef NTTMUL_HOOK_TW
#define NTTMUL_HOOK_TW(tw, idx, dir) ((tw)[idx])
#endif
#ifndef NTTMUL_HOOK_XCHG
#define NTTMUL_HOOK_XCHG() do { } while (0)
#endif
#if defined(NTTMUL_HOOK_COLS_LD) || defined(NTTMUL_HOOK_COLS_ST)
#define NTTMUL_COLS_HOOKED 1  // (kbench pricing builds: the column passes keep global addressing)
#else
#define NTTMUL_COLS_HOOKED 0
#endif
#ifndef NTTMUL_HOOK_COLS_LD
#define NTTMUL_HOOK_COLS_LD(base, p, sh, col, dir) (base)
#endif
#ifndef NTTMUL_HOOK_COLS_ST
#define NTTMUL_HOOK_COLS_ST(base, p, sh, col) (base)
#endif

namespace nttmul {

template <class W>
__host__ __device__ constexpr int lds_regions() { return sizeof(W) == 8 ? 1 : NTTMUL_LDS_REGIONS; }

template <class A>
struct KParams {
  A ar;
  const TwPair<typename A::word> *fw;  // forward twiddles  (mixed_powers_rev + Shoup)
  const TwPair<typename A::word> *iw;  // inverse twiddles  (inv_mixed_powers_rev + Shoup)
  typename A::word f, fs;              // F  = n^-1 R mod q (R = Montgomery radix)
  typename A::word wf, wfs;            // iw[1] * F mod q
};

// Dry run of the product dispatch (describe_polymul -> nttmul_kernel_name): while tl_describe is
// set, the launchers append the kernels they would launch to it and launch nothing, so the name
// the bench reports comes from the same dispatch code that runs.
static thread_local std::string *tl_describe = nullptr;
template <class A> struct AName;
template <class T> constexpr const char *word_name() { return sizeof(T) == 8 ? "u64" : "u32"; }
static void describe_add(const std::string &k) {
  if (!tl_describe->empty()) *tl_describe += " + ";
  *tl_describe += k;
}

// ---------------------------------------------------------------------------------------------
// Layout algebra of the register groups (all compile-time except the per-thread base)
// ---------------------------------------------------------------------------------------------
// WT (wave-typed layouts, n = 4096 rows of the Plantard kernels, NTTMUL_WAVE_TYPED): groups 1
// and 2 take their element bits from the thread index in another order, so that the bit that
// says whether the previous group's last forward stage wrote an element as a sum or as a
// difference (element bit 8 after group 0, bit 4 after group 1) is thread bit 6 -- the same for
// a whole wave.  Those last stages can then leave their differences signed across the LDS
// exchange (one instruction less per butterfly, -0.85 % time by ablation, profiles/r3/c3/) and
// the next group's first stage picks its operand type with one wave-uniform branch.  Group 1:
// thread bits 0-3 -> element bits 0-3, 4 -> 9, 5 -> 10, 6 -> 8, 7 -> 11; group 2: thread bits
// 0-5 -> element bits 5-10, 6 -> 4, 7 -> 11.  Both exchanges then pad e + (e >> 5), which the bank
// census (tests/test_layout.py) finds conflict-free for both layouts of each exchange.
// (NTTMUL_WAVE_TYPED: arith_select.hpp, shared with the planner's twiddle forms)
template <int LOGS, bool WT = false>
struct Groups {
  static_assert(!WT || LOGS == 12, "wave-typed layouts are defined for 4096-coefficient rows");
  static constexpr int N = 1 << LOGS;
  static constexpr int G = (LOGS + 3) / 4;
  static constexpr int S(int g) { return LOGS / G + (g < LOGS % G ? 1 : 0); }
  static constexpr int ST0(int g) {
    int s = 0;
    for (int i = 0; i < g; i++) s += S(i);
    return s;
  }
  static constexpr int NS(int g) { return 16 >> S(g); }         // independent sets per thread
  static constexpr int LR(int g) { return LOGS - ST0(g) - S(g); } // log2 of the group's min distance
  static constexpr int LNS(int g) { return 4 - S(g); }
  // element index = base(g, j) + off(g, k), with base and off bit-disjoint (so the LDS pad
  // e + (e >> 4) also splits into a per-thread part and an immediate offset).
  static constexpr int off(int g, int k) {
    int ns = NS(g), lr = LR(g), s = S(g);
    int m = k / ns, sidx = k % ns;
    if (lr >= LNS(g)) return sidx + (m << lr);
    return ((sidx >> lr) << (lr + s)) + (sidx & ((1 << lr) - 1)) + (m << lr);
  }
  __host__ __device__ static constexpr int base_wt(int g, int j) {
    return g == 1 ? (j & 15) + (((j >> 4) & 1) << 9) + (((j >> 5) & 1) << 10) +
                        (((j >> 6) & 1) << 8) + (((j >> 7) & 1) << 11)
                  : ((j & 63) << 5) + (((j >> 6) & 1) << 4) + (((j >> 7) & 1) << 11);
  }
  // WT: the operand type (0 sum, 1 difference) of the elements a thread holds at the start of
  // register group g >= 1; thread bit 6, uniform over the wave
  __device__ static __forceinline__ int wave_type(int j) {
    return __builtin_amdgcn_readfirstlane((j >> 6) & 1);
  }
  __device__ static __forceinline__ int base(int g, int j) {
    if (WT && g > 0) return base_wt(g, j);
    int lr = LR(g), s = S(g), lns = LNS(g);
    if (lr >= lns) {
      int set0 = j << lns;
      return ((set0 >> lr) << (lr + s)) + (set0 & ((1 << lr) - 1));
    }
    return j << 4;
  }
  // block index of register k's set (twiddle index contribution), B = set >> lr
  __device__ static __forceinline__ int blk(int g, int j, int k) {
    int lr = LR(g), lns = LNS(g);
    int sidx = k % NS(g);
    if (g == 0) return 0;
    if (WT) return base_wt(g, j) >> (lr + S(g));  // the element bits above the group's stages
    if (lr >= lns) return (j << lns) >> lr;
    return (j << (lns - lr)) + (sidx >> lr);
  }
  // register holding element offset o in group g's layout (inverse of off)
  static constexpr int reg_of(int g, int o) {
    for (int k = 0; k < 16; k++)
      if (off(g, k) == o) return k;
    return -1;
  }
  // LDS padding of exchange X (between register groups X and X + 1): e + ((e >> s) << t), linear
  // over bit-disjoint parts (so pad(base + off) = pad(base) + pad(off) and off stays an
  // immediate offset).  Chosen per exchange by a bank census of both register layouts it
  // connects (32 banks per 32-lane group): group 0 hands each lane consecutive
  // elements across the wave, which e + (e >> 4) 2-way conflicts (every 32 consecutive words span
  // 34); e + ((e >> (LOGS - 4)) << (LOGS - 8)) keeps those lanes on distinct banks and still
  // separates group 1's two 16-element halves.  Exchange 1 (groups 1 <-> 2) keeps e + (e >> 4).
  // n = 1024 and 512 (one wave per product, three groups of 3-4 stages) take a second term,
  // e + ((e >> s) << t) + ((e >> s2) << t2), found by the same census (tests/test_layout.py): the
  // single-term pads left 32 extra cycles on each exchange at n = 1024 (PMC: 33 % of LDS cycles)
  static constexpr bool kPad0 = NTTMUL_PAD0 && LOGS >= 10 && G > 2;
  static constexpr bool kPad2 = NTTMUL_PAD0 && NTTMUL_PAD2 && (LOGS == 10 || LOGS == 9);
  static constexpr int PS(int x) {
    return WT ? 5
              : kPad2 ? (LOGS == 10 ? (x == 0 ? 6 : 4) : (x == 0 ? 5 : 4))
                      : (x == 0 && kPad0 ? LOGS - 4 : 4);
  }
  static constexpr int PT(int x) {
    return WT ? 0
              : kPad2 ? (LOGS == 10 ? (x == 0 ? 3 : 1) : (x == 0 ? 0 : 1))
                      : (x == 0 && kPad0 ? LOGS - 8 : 0);
  }
  static constexpr int PS2(int x) { return kPad2 ? (LOGS == 10 ? 8 : (x == 0 ? 7 : 8)) : 31; }
  template <int X>
  static constexpr int padx(int e) { return e + ((e >> PS(X)) << PT(X)) + (e >> PS2(X)); }
  static constexpr int pad(int e) { return padx<1>(e); }
  // padded LDS words per polynomial (>= every padx + 1; the pads are increasing in e)
  static constexpr int NP = (padx<0>(N - 1) > padx<1>(N - 1) ? padx<0>(N - 1) : padx<1>(N - 1)) + 1 >
                                    N + N / 16
                                ? (padx<0>(N - 1) > padx<1>(N - 1) ? padx<0>(N - 1) : padx<1>(N - 1)) + 1
                                : N + N / 16;
};

template <int LOGS>
constexpr bool groups_agree() {
  for (int g = 0; g < Groups<LOGS>::G; g++)
    if (Groups<LOGS>::S(g) != groups_s(LOGS, g)) return false;
  return Groups<LOGS>::G == groups_g(LOGS);
}
static_assert(groups_agree<8>() && groups_agree<9>() && groups_agree<10>() && groups_agree<11>() &&
                  groups_agree<12>(),
              "arith_select.hpp's group helpers (planner twiddle forms) must match Groups<>");

template <class W, class T>
__device__ __forceinline__ W to_word(T v) { return (W)v; }

// Arith32P's typed CT (modarith.hpp Arith32P::ct<XC, XN, YN>)
template <class A>
struct IsPlantard : std::false_type {};
template <>
struct IsPlantard<Arith32P> : std::true_type {};
template <>
struct IsPlantard<Arith32P3> : std::true_type {};
template <> struct AName<Arith32> { static constexpr const char *v = "Arith32"; };
template <> struct AName<Arith32H> { static constexpr const char *v = "Arith32H"; };
template <> struct AName<Arith32P> { static constexpr const char *v = "Arith32P"; };
template <> struct AName<Arith32P3> { static constexpr const char *v = "Arith32P3"; };
template <> struct AName<Arith32W> { static constexpr const char *v = "Arith32W"; };
template <> struct AName<Arith64> { static constexpr const char *v = "Arith64"; };
template <class A>
__host__ __device__ constexpr bool kTypedP() {
  if constexpr (IsPlantard<A>::value) return A::kTypedP;
  return false;
}
// wave-typed layouts (Groups WT) for the typed Plantard kernels' 4096-coefficient rows; the
// planner stores the matching twiddle forms (arith_select.hpp p_signed_fw_entry)
template <class A, int LOGS>
__host__ __device__ constexpr bool kWT() {
  return wave_typed_rows(LOGS) && kTypedP<A>() && NTTMUL_P_TYPED >= 2;
}

// Coefficient streams are touched once per product: NTTMUL_NT marks them non-temporal.  The row
// pass of a multi-pass product (L1 > 0) reads and writes intermediates that the column passes
// touch again, so NTTMUL_NT_MP (default 0) keeps those accesses temporal: a sub-batch whose
// scratch fits the Infinity Cache can then stay there between the three launches.
#ifndef NTTMUL_NT_MP
#define NTTMUL_NT_MP 0
#endif
// column passes of the multi-pass product through non-temporal loads / stores: C5 1.375-1.383
// vs 1.417-1.434 ms (kbench A/B, identical checksums, profiles/r2/nt_cols/); the row pass
// keeps its intermediates temporal (NTTMUL_NT_MP = 1 measured 1.400 ms)
#ifndef NTTMUL_NT_COLS
#define NTTMUL_NT_COLS 1
#endif
template <bool NT, class T>
__device__ __forceinline__ T ld_stream(const T *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT, class T>
__device__ __forceinline__ void st_stream(T *p, T v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// Buffer-resource streams (NTTMUL_CPOL): a descriptor over one block-uniform span of words and
// 32-bit per-lane byte offsets; AUX = the cache-policy bits of the load / store
template <class T>
__device__ __forceinline__ auto span_rsrc(const T *p, size_t words) {
  return __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, (int)(words * sizeof(T)), 0x00020000);
}
// SOFF: a wave-uniform byte offset passed as the instruction's scalar offset (NTTMUL_BUF_SOFF:
// the register's constant part, so the per-lane offset is the thread's base alone and no VALU
// add / or forms each register's address)
template <int AUX, class R>
__device__ __forceinline__ uint32_t buf_ld32(R r, int byte_off, int soff = 0) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, soff, AUX);
}
template <int AUX, class R>
__device__ __forceinline__ void buf_st32(R r, int byte_off, uint32_t v, int soff = 0) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, byte_off, soff, AUX);
}
#ifndef NTTMUL_BUF_SOFF
#define NTTMUL_BUF_SOFF 1
#endif
template <int AUX, class R>
__device__ __forceinline__ uint64_t buf_ld64(R r, int byte_off, int soff) {
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  const u2 v = __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, soff, AUX);
  return ((uint64_t)v.y << 32) | v.x;
}
template <int AUX, class R>
__device__ __forceinline__ void buf_st64(R r, int byte_off, uint64_t v, int soff) {
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  const u2 w = {(unsigned)v, (unsigned)(v >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(w, r, byte_off, soff, AUX);
}
// The square split's column passes (k_cols8, 64-bit words) through buffer instructions on a
// descriptor per polynomial (block-uniform) with 32-bit lane offsets and each register's constant
// offset in the scalar offset, instead of a 64-bit address per register (NTTMUL_C5_BUF; with the
// row pass in the same form: C5 1.221 vs 1.243 ms, kbench A/B interleaved, identical checksums,
// profiles/r6/ab_c5_buf.json)
#ifndef NTTMUL_C5_BUF
#define NTTMUL_C5_BUF 1
#endif

// One forward CT stage l of group g on NPOLY (1 or 2) polynomials (same twiddles); the twiddles
// of the group's last performed stage are kept in zw[X register] (see base_mult).  TIN: under the
// wave-typed layouts (kWT) the operand type of the first stage of groups g >= 1, chosen by the
// caller's wave-uniform branch (1: the previous group's differences, left signed).
template <class A, int LOGS, int g, int NPOLY, int SKIP, int TIN>
__device__ __forceinline__ void fwd_stage(const A &ar, typename A::word (&x)[16],
                                          typename A::word (&y)[16],
                                          const TwPair<typename A::word> *__restrict__ tw, int j,
                                          int row, int l1, TwPair<typename A::word> (&zw)[16],
                                          int l) {
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int S = Gr::S(g), st0 = Gr::ST0(g), ns = Gr::NS(g);
  const int dist = 8 >> l;
  const int st = st0 + l;
  const int tbase = (1 << (l1 + st)) + (row << st);
#pragma unroll
  for (int k = 0; k < 16; k++) {
    if (k & dist) continue;
    const int m = k / ns;
    const int idx = tbase + (Gr::blk(g, j, k) << l) + (m >> (S - l));
    if constexpr (A::kTyped) {
      // operand type: bit 2 dist of k says the previous stage of this group wrote it as Y
      // (N-type); the group's first stage reads P-type; its last writes P-type
      const bool in_n = l > 0 && (k & (2 * dist));
      const bool out_p = l == S - SKIP - 1;
      const TwPair<typename A::word> t = in_n ? tw[idx + (1 << (l1 + LOGS))] : tw[idx];
      if (out_p) zw[k] = t;
      const bool xc = NTTMUL_FIRST_XC && g == 0 && l == 0 && l1 == 0;
#define NTTMUL_CT_T(IN, OUT, XC_)                                 \
  do {                                                            \
    ar.template ct_t<IN, OUT, XC_>(x[k], x[k + dist], t.w, t.ws); \
    if (NPOLY == 2) ar.template ct_t<IN, OUT, XC_>(y[k], y[k + dist], t.w, t.ws); \
  } while (0)
      if (xc) {
        if (out_p) NTTMUL_CT_T(false, true, true); else NTTMUL_CT_T(false, false, true);
      } else if (in_n) {
        if (out_p) NTTMUL_CT_T(true, true, false); else NTTMUL_CT_T(true, false, false);
      } else {
        if (out_p) NTTMUL_CT_T(false, true, false); else NTTMUL_CT_T(false, false, false);
      }
#undef NTTMUL_CT_T
      continue;
    }
    const TwPair<typename A::word> t = NTTMUL_HOOK_TW(tw, idx, 0);
    if (l == S - SKIP - 1) zw[k] = t;
    if constexpr (kTypedP<A>()) {
      // Arith32P: register k was written as a (signed) difference by the previous stage iff
      // bit 2 dist is set; this stage leaves its difference in k + dist signed iff the next
      // stage of the group uses that register as an X (bit dist / 2 clear).  kWT: the first
      // stage of groups 1 and 2 reads the type TIN of the wave
      constexpr bool kWt = kWT<A, LOGS>();
      const bool xn = l > 0 ? (k & (2 * dist)) != 0 : (kWt && g > 0 && TIN);
      // (P_TYPED 2: the last stage before the base multiplication leaves its differences
      // signed as well; Arith32P::basemul corrects the -w blocks with the carry of x + q; kWT:
      // so does the last stage before an exchange)
      const bool yn = (NTTMUL_P_TYPED >= 2
                           ? l < S - SKIP - 1 || (SKIP > 0 && g + 1 == Gr::G) ||
                                 (kWt && g + 1 < Gr::G)
                           : l < S - SKIP - 1 && !((k + dist) & (dist >> 1)));
      const bool xc = NTTMUL_FIRST_XC && g == 0 && l == 0 && l1 == 0;
      constexpr bool kAsm = kWt && g > 0 && TIN;  // see Arith32P::pmul_s
#define NTTMUL_CT_P(XC_, XN_, YN_)                                         \
  do {                                                                     \
    ar.template ct<XC_, XN_, YN_, kAsm>(x[k], x[k + dist], t.w, t.ws);      \
    if (NPOLY == 2) ar.template ct<XC_, XN_, YN_, kAsm>(y[k], y[k + dist], t.w, t.ws); \
  } while (0)
      if (xc) {
        if (yn) NTTMUL_CT_P(true, false, true); else NTTMUL_CT_P(true, false, false);
      } else if (xn) {
        if (yn) NTTMUL_CT_P(false, true, true); else NTTMUL_CT_P(false, true, false);
      } else {
        if (yn) NTTMUL_CT_P(false, false, true); else NTTMUL_CT_P(false, false, false);
      }
#undef NTTMUL_CT_P
      continue;
    }
    // global stage 0 of a whole polynomial reads canonical input (the API contract, [0, q)):
    // its X operands need no reduction
    if (NTTMUL_FIRST_XC && g == 0 && l == 0 && l1 == 0) {
      ar.template ct<true>(x[k], x[k + dist], t.w, t.ws);
      if (NPOLY == 2) ar.template ct<true>(y[k], y[k + dist], t.w, t.ws);
    } else {
      ar.ct(x[k], x[k + dist], t.w, t.ws);
      if (NPOLY == 2) ar.ct(y[k], y[k + dist], t.w, t.ws);
    }
  }
}

// Forward CT stages of group g on NPOLY (1 or 2) polynomials (same twiddles).  SKIP: leave out
// the last SKIP stages of the group (the incomplete transform of the product kernel, see
// base_mult).
template <class A, int LOGS, int g, int NPOLY = 2, int SKIP = 0, int L = 0>
__device__ __forceinline__ void fwd_group(const A &ar, typename A::word (&x)[16],
                                          typename A::word (&y)[16],
                                          const TwPair<typename A::word> *__restrict__ tw, int j,
                                          int row, int l1,
                                          TwPair<typename A::word> (&zw)[16]) {
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int S = Gr::S(g);
  if constexpr (sizeof(typename A::word) == 8) {
    // 64-bit words: stages by compile-time recursion.  The loop body exceeds the unroller's
    // threshold, and a rolled loop turns every register index into a runtime one (s_set_gpr_idx
    // moves and per-register branches): C5 1.42 -> 1.36 ms (profiles/r3/c5/unroll_ab.txt).  (The
    // 32-bit kernels unroll either way; the recursion reorders them for +0.2-0.8 %, so they keep
    // the loop.)
    if constexpr (L < S - SKIP) {
      fwd_stage<A, LOGS, g, NPOLY, SKIP, 0>(ar, x, y, tw, j, row, l1, zw, L);
      fwd_group<A, LOGS, g, NPOLY, SKIP, L + 1>(ar, x, y, tw, j, row, l1, zw);
    }
  } else {
#pragma unroll
    for (int l = 0; l < S - SKIP; l++) {
      if (kWT<A, LOGS>() && g > 0 && l == 0) {  // one wave-uniform branch per group
        if (Gr::wave_type(j))
          fwd_stage<A, LOGS, g, NPOLY, SKIP, 1>(ar, x, y, tw, j, row, l1, zw, l);
        else
          fwd_stage<A, LOGS, g, NPOLY, SKIP, 0>(ar, x, y, tw, j, row, l1, zw, l);
      } else {
        fwd_stage<A, LOGS, g, NPOLY, SKIP, 0>(ar, x, y, tw, j, row, l1, zw, l);
      }
    }
  }
}

// One inverse GS stage l of group g.  SCALE: fold F into the global stage 0.  SKIP: the group's
// last SKIP forward stages were left out (the first SKIP inverse ones).
template <class A, int LOGS, int g, bool SCALE, int SKIP>
__device__ __forceinline__ void inv_stage(const KParams<A> &P, typename A::word (&x)[16],
                                          const TwPair<typename A::word> *__restrict__ tw, int j,
                                          int row, int l1, int l) {
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int S = Gr::S(g), st0 = Gr::ST0(g), ns = Gr::NS(g);
  const int dist = 8 >> l;
  const int st = st0 + l;
  const int tbase = (1 << (l1 + st)) + (row << st);
#pragma unroll
  for (int k = 0; k < 16; k++) {
    if (k & dist) continue;
    if constexpr (A::kTyped) {
      // first stage of the group (inverse order) reads P-type; later ones read the previous
      // stage's Y registers (bit dist / 2 of k) as N-type; the group's last stage writes P-type
      const bool in_n = l < S - 1 - SKIP && (k & (dist >> 1));
      const bool out_p = l == 0;
      if (SCALE && st == 0) {
        if (in_n)
          P.ar.template gs_scaled_t<true>(x[k], x[k + dist], P.f, P.fs, P.wf, P.wfs);
        else
          P.ar.template gs_scaled_t<false>(x[k], x[k + dist], P.f, P.fs, P.wf, P.wfs);
        continue;
      }
      const int m = k / ns;
      const int idx = tbase + (Gr::blk(g, j, k) << l) + (m >> (S - l));
      const TwPair<typename A::word> t = out_p ? tw[idx] : tw[idx + (1 << (l1 + LOGS))];
      if (in_n) {
        if (out_p) P.ar.template gs_t<true, true>(x[k], x[k + dist], t.w, t.ws);
        else P.ar.template gs_t<true, false>(x[k], x[k + dist], t.w, t.ws);
      } else {
        if (out_p) P.ar.template gs_t<false, true>(x[k], x[k + dist], t.w, t.ws);
        else P.ar.template gs_t<false, false>(x[k], x[k + dist], t.w, t.ws);
      }
      continue;
    }
    if (SCALE && st == 0) {
      P.ar.gs_scaled(x[k], x[k + dist], P.f, P.fs, P.wf, P.wfs);
    } else {
      const int m = k / ns;
      const int idx = tbase + (Gr::blk(g, j, k) << l) + (m >> (S - l));
      const TwPair<typename A::word> t = NTTMUL_HOOK_TW(tw, idx, 1);
      P.ar.gs(x[k], x[k + dist], t.w, t.ws);
    }
  }
}

// Inverse GS stages of group g (reverse stage order); 64-bit words by compile-time recursion over
// L (see fwd_group).
template <class A, int LOGS, int g, bool SCALE, int SKIP = 0, int L = Groups<LOGS>::S(g) - 1 - SKIP>
__device__ __forceinline__ void inv_group(const KParams<A> &P, typename A::word (&x)[16],
                                          const TwPair<typename A::word> *__restrict__ tw, int j,
                                          int row, int l1) {
  if constexpr (sizeof(typename A::word) == 8) {
    if constexpr (L >= 0) {
      inv_stage<A, LOGS, g, SCALE, SKIP>(P, x, tw, j, row, l1, L);
      inv_group<A, LOGS, g, SCALE, SKIP, L - 1>(P, x, tw, j, row, l1);
    }
  } else {
#pragma unroll
    for (int l = L; l >= 0; l--) inv_stage<A, LOGS, g, SCALE, SKIP>(P, x, tw, j, row, l1, l);
  }
}

// LDS ordering between an exchange's writes and reads: the whole workgroup (SYNC 0), or only the
// wave (SYNC 1: a wave owns its product and its LDS region; a wave's LDS operations execute in
// order, so only the compiler must be kept from moving them)
template <int SYNC>
__device__ __forceinline__ void xsync() {
  if constexpr (SYNC == 0) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}


// Move 16 registers of each region from layout gfrom to layout gto through LDS.  ES: LDS words
// between consecutive (padded) elements of one polynomial (1; k_cols8 interleaves the 16 column
// transforms of a workgroup element by element, ES = 16, so a wave's lanes on adjacent columns
// touch adjacent words).
template <int LOGS, int gfrom, int gto, int NREG, class W, int SYNC = 0, bool WT = false, int ES = 1>
__device__ __forceinline__ void exchange(W (&x)[16], W (&y)[16], W *lds_x, W *lds_y, int j) {
  using Gr = Groups<LOGS, WT>;
  NTTMUL_HOOK_XCHG();
  constexpr int X = gfrom < gto ? gfrom : gto;
  const int bw = Gr::template padx<X>(Gr::base(gfrom, j)) * ES;
  const int br = Gr::template padx<X>(Gr::base(gto, j)) * ES;
  if (lds_regions<W>() == 1 && NREG == 2) {  // one region, the two polynomials in turn
#pragma unroll
    for (int k = 0; k < 16; k++) lds_x[bw + Gr::template padx<X>(Gr::off(gfrom, k)) * ES] = x[k];
    xsync<SYNC>();
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = lds_x[br + Gr::template padx<X>(Gr::off(gto, k)) * ES];
    xsync<SYNC>();
#pragma unroll
    for (int k = 0; k < 16; k++) lds_x[bw + Gr::template padx<X>(Gr::off(gfrom, k)) * ES] = y[k];
    xsync<SYNC>();
#pragma unroll
    for (int k = 0; k < 16; k++) y[k] = lds_x[br + Gr::template padx<X>(Gr::off(gto, k)) * ES];
    xsync<SYNC>();
    return;
  }
#pragma unroll
  for (int k = 0; k < 16; k++) {
    lds_x[bw + Gr::template padx<X>(Gr::off(gfrom, k)) * ES] = x[k];
    if (NREG == 2) lds_y[bw + Gr::template padx<X>(Gr::off(gfrom, k)) * ES] = y[k];
  }
  xsync<SYNC>();
#pragma unroll
  for (int k = 0; k < 16; k++) {
    x[k] = lds_x[br + Gr::template padx<X>(Gr::off(gto, k)) * ES];
    if (NREG == 2) y[k] = lds_y[br + Gr::template padx<X>(Gr::off(gto, k)) * ES];
  }
  xsync<SYNC>();
}

template <class A, int LOGS, int g, int NPOLY = 2, int SKIP = 0, int SYNC = 0, int ES = 1>
__device__ __forceinline__ void fwd_all(const A &ar, typename A::word (&x)[16],
                                        typename A::word (&y)[16], typename A::word *lx,
                                        typename A::word *ly,
                                        const TwPair<typename A::word> *__restrict__ tw, int j,
                                        int row, int l1, TwPair<typename A::word> (&zw)[16]) {
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr bool last = g + 1 == Gr::G;
  fwd_group<A, LOGS, g, NPOLY, last ? SKIP : 0>(ar, x, y, tw, j, row, l1, zw);
  if constexpr (!last) {
    exchange<LOGS, g, g + 1, NPOLY, typename A::word, SYNC, kWT<A, LOGS>(), ES>(x, y, lx, ly, j);
    fwd_all<A, LOGS, g + 1, NPOLY, SKIP, SYNC, ES>(ar, x, y, lx, ly, tw, j, row, l1, zw);
  }
}

// NPOLY 2 (standalone inverse transforms, k_xform): y is a second polynomial inverted alongside x
// with the same twiddles (the product inverts one)
template <class A, int LOGS, int g, bool SCALE, int SKIP = 0, int SYNC = 0, int NPOLY = 1,
          int ES = 1>
__device__ __forceinline__ void inv_all(const KParams<A> &P, typename A::word (&x)[16],
                                        typename A::word (&y)[16], typename A::word *lx,
                                        typename A::word *ly,
                                        const TwPair<typename A::word> *__restrict__ tw, int j,
                                        int row, int l1) {
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  inv_group<A, LOGS, g, SCALE, g + 1 == Gr::G ? SKIP : 0>(P, x, tw, j, row, l1);
  if constexpr (NPOLY == 2) inv_group<A, LOGS, g, SCALE, g + 1 == Gr::G ? SKIP : 0>(P, y, tw, j, row, l1);
  if constexpr (g > 0) {
    exchange<LOGS, g, g - 1, NPOLY, typename A::word, SYNC, kWT<A, LOGS>(), ES>(x, y, lx, ly, j);
    inv_all<A, LOGS, g - 1, SCALE, SKIP, SYNC, NPOLY, ES>(P, x, y, lx, ly, tw, j, row, l1);
  }
}

// Incomplete-transform product (Kyber-style): the last D forward stages, the pointwise product
// and the first D inverse stages are replaced by products in Z_q[x]/(x^(2^D) - z) of the 2^D-
// coefficient blocks the truncated forward transform leaves.  The CT butterfly with twiddle w
// splits x^(2d) - w^2 into (x^d - w)(x^d + w), so a block that was the X (Y) output of the last
// performed stage is a residue mod x^(2^D) - w (x^(2^D) + w): z = +-w, the twiddle already in
// zw.  The last group always starts at a multiple of 16 elements, so bit D of a register's
// offset says X or Y.  Same canonical output as the full transform (the product is unique).
//
// base_mult_rec: the same with the blocks by compile-time recursion over the register index K0
// instead of an unrolled loop, for Arith32P3 (NTTMUL_P3_PIN; base_mult below dispatches to it):
// its base multiplication pins the halfway fold with an empty asm, and a loop holding inline asm
// is not fully unrolled (its register indices turn into runtime ones).  The other classes keep
// the loop (for them the recursion only reorders the code: +15 VALU in the C5 row pass).
template <class A, int LOGS, int D, int K0 = 0>
__device__ __forceinline__ void base_mult_rec(const A &ar, typename A::word (&x)[16],
                                          const typename A::word (&y)[16],
                                          const TwPair<typename A::word> (&zw)[16], int j) {
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int g = Gr::G - 1, B = 1 << D;
  static_assert(D > 0 && Gr::S(g) > D, "base blocks of 2^D > 1 coefficients in the last group");
  if constexpr (K0 < 16) {
    constexpr int o0 = Gr::off(g, K0);
    if constexpr ((o0 & (B - 1)) == 0) {  // K0 holds a block's constant coefficient
      int r[B];
#pragma unroll
      for (int i = 0; i < B; i++) r[i] = Gr::reg_of(g, o0 + i);
      constexpr bool neg = (o0 >> D) & 1;
      constexpr int kz = Gr::reg_of(g, o0 & ~B);
      TwPair<typename A::word> z = zw[kz];
      // typed arithmetic: the last forward stage (dist 8 >> (S - D - 1)) multiplied N-type
      // operands, and so kept the centred twiddle, when bit 2 dist of its X register is set
      constexpr int dl = 8 >> (Gr::S(g) - D - 1);
      // (Arith32P, NTTMUL_P_TYPED 2: the same condition says the pair is in signed form)
      constexpr bool typed_z = A::kTyped || (kTypedP<A>() && NTTMUL_P_TYPED >= 2);
      // (kWT, when that stage was its group's first: the pair is in signed form exactly when the
      // wave's elements were the previous group's differences.  The signed-input product is
      // exact for canonical inputs too, so every wave takes it: the unsigned pair of the other
      // waves becomes the signed one by b1 + (b0 >> 31), two instructions, instead of a second
      // copy of the base multiplication behind a branch)
      constexpr bool kWtFirst = kWT<A, LOGS>() && Gr::S(g) - D - 1 == 0;
      if constexpr (kWtFirst)
        z.ws += (typename A::word)((z.w >> 31) & (1 - Gr::wave_type(j)));
      constexpr bool zc = typed_z && (kWtFirst || (Gr::S(g) - D - 1 > 0 && (kz & (2 * dl))));
      typename A::word a[B], b[B];
#pragma unroll
      for (int i = 0; i < B; i++) a[i] = x[r[i]], b[i] = y[r[i]];
      ar.template basemul<B, neg, zc>(a, b, z.w, z.ws);
#pragma unroll
      for (int i = 0; i < B; i++) x[r[i]] = a[i];
    }
    base_mult_rec<A, LOGS, D, K0 + 1>(ar, x, y, zw, j);
  }
}

template <class A, int LOGS, int D>
__device__ __forceinline__ void base_mult(const A &ar, typename A::word (&x)[16],
                                          const typename A::word (&y)[16],
                                          const TwPair<typename A::word> (&zw)[16], int j) {
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int g = Gr::G - 1, B = 1 << D;
  static_assert(D == 0 || Gr::S(g) > D, "last register group too short for the base blocks");
  if constexpr (D == 0) {
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = ar.mont(x[k], y[k]);
  } else if constexpr (std::is_same<A, Arith32P3>::value && NTTMUL_P3_PIN) {
    base_mult_rec<A, LOGS, D>(ar, x, y, zw, j);
  } else {
#pragma unroll
    for (int k0 = 0; k0 < 16; k0++) {
      const int o0 = Gr::off(g, k0);
      if (o0 & (B - 1)) continue;  // k0 holds a block's constant coefficient
      int r[B];
#pragma unroll
      for (int i = 0; i < B; i++) r[i] = Gr::reg_of(g, o0 + i);
      const bool neg = (o0 >> D) & 1;
      const int kz = Gr::reg_of(g, o0 & ~B);
      TwPair<typename A::word> z = zw[kz];
      // typed arithmetic: the last forward stage (dist 8 >> (S - D - 1)) multiplied N-type
      // operands, and so kept the centred twiddle, when bit 2 dist of its X register is set
      constexpr int dl = 8 >> (Gr::S(g) - D - 1);
      // (Arith32P, NTTMUL_P_TYPED 2: the same condition says the pair is in signed form)
      constexpr bool typed_z = A::kTyped || (kTypedP<A>() && NTTMUL_P_TYPED >= 2);
      // (kWT, when that stage was its group's first: the pair is in signed form exactly when the
      // wave's elements were the previous group's differences.  The signed-input product is
      // exact for canonical inputs too, so every wave takes it: the unsigned pair of the other
      // waves becomes the signed one by b1 + (b0 >> 31), two instructions, instead of a second
      // copy of the base multiplication behind a branch)
      constexpr bool kWtFirst = kWT<A, LOGS>() && Gr::S(g) - D - 1 == 0;
      if constexpr (kWtFirst)
        z.ws += (typename A::word)((z.w >> 31) & (1 - Gr::wave_type(j)));
      const bool zc = typed_z && (kWtFirst || (Gr::S(g) - D - 1 > 0 && (kz & (2 * dl))));
      typename A::word a[B], b[B];
#pragma unroll
      for (int i = 0; i < B; i++) a[i] = x[r[i]], b[i] = y[r[i]];
      if (zc) {
        if (neg)
          ar.template basemul<B, true, true>(a, b, z.w, z.ws);
        else
          ar.template basemul<B, false, true>(a, b, z.w, z.ws);
      } else if (neg)
        ar.template basemul<B, true>(a, b, z.w, z.ws);
      else
        ar.template basemul<B, false>(a, b, z.w, z.ws);
#pragma unroll
      for (int i = 0; i < B; i++) x[r[i]] = a[i];
    }
  }
}

// Threads per k_rows workgroup: 256 (one n = 4096 product, or 256 / (n / 16) smaller ones),
// except one wave per workgroup at n = 1024 (NTTMUL_SMALL_BLOCK): one product per wave, so no
// barrier ties four independent products together.  C2 (n = 1024 x 4096) 22.2 -> 21.6 us,
// n = 1024 x 262144 -1 %; n = 256 one wave per 4 products was not faster (profiles/r2)
#ifndef NTTMUL_SMALL_BLOCK
#define NTTMUL_SMALL_BLOCK 1
#endif
__host__ __device__ constexpr int rows_threads(int logs) {
  return NTTMUL_SMALL_BLOCK && logs == 10 ? 64 : 256;
}
// __launch_bounds__ minimum waves per SIMD of k_rows: NTTMUL_MIN_WAVES, and for the one-wave
// n = 1024 products NTTMUL_MIN_WAVES_1024 (an A/B switch: 8 gives 64 VGPRs instead of 84-86, so
// the next C2 launch's four waves per SIMD fit beside the running four on another stream, but
// measured +3.2 % on one stream and +3.6 % on two; default: no bound)
#ifndef NTTMUL_MIN_WAVES_1024
#define NTTMUL_MIN_WAVES_1024 NTTMUL_MIN_WAVES
#endif
__host__ __device__ constexpr int rows_min_waves(int logs) {
  return NTTMUL_SMALL_BLOCK && logs == 10 ? NTTMUL_MIN_WAVES_1024 : NTTMUL_MIN_WAVES;
}
// Square split (k_cols8): the intermediates ta, tb, tc tiled per 16 columns (NTTMUL_C5_TILE), so
// the column passes store / load one contiguous 32 KiB tile per workgroup and the row pass moves
// 512 contiguous bytes per instruction, instead of 128-byte runs 2 KiB apart (a row-major
// column) on the column side
#ifndef NTTMUL_C5_TILE
#define NTTMUL_C5_TILE 1
#endif
__host__ __device__ constexpr bool c8_tile(int logs, int l1) {
  return NTTMUL_C5_TILE && logs == 8 && l1 == 8;
}

// Fused product of `units` independent rows of 2^LOGS coefficients.
//   L1 == 0 : each unit is a whole polynomial (n = 2^LOGS): full product, canonical output.
//   L1 >  0 : unit u is row (u mod 2^L1) of polynomial (u >> L1) after the column pass; the
//             row's stages are global stages L1 .. L1+LOGS-1; output stays lazy in [0, 2q).

// In-kernel clock (lib/libnttmul_diag.so only, built with NTTMUL_CLOCK_STAMPS; MI355X_MICROARCH.md
// 'DVFS give-back' item 6): thread 0 of each k_rows workgroup stamps s_memtime (shader clock) and
// s_memrealtime (100 MHz) at entry and after issuing its stores, into a buffer of its own that no
// other code reads; the workgroup's clock is d(memtime) / d(realtime) x 100 MHz.  The product
// kernels of libnttmul.so execute no stamp.
#ifdef NTTMUL_CLOCK_STAMPS
constexpr unsigned kClkSlots = 1u << 16;
__device__ unsigned long long g_clk[kClkSlots * 4];
hipError_t read_clock_stamps(void *dst, size_t blocks) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_clk),
                             (blocks < kClkSlots ? blocks : kClkSlots) * 4 * sizeof(unsigned long long));
}
__device__ __forceinline__ void clk_stamp(int k) {
  if (threadIdx.x == 0) {
    unsigned long long t, r;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t), "=s"(r)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long *p = g_clk + (blockIdx.x % kClkSlots) * 4 + 2 * k;
    p[0] = t;
    p[1] = r;
  }
}
#define CLK_STAMP(k) clk_stamp(k)
#else
#define CLK_STAMP(k) do { } while (0)
#endif

template <class A, class TIn, class TOut, int LOGS, int L1, bool PRIO = false>
__global__ __launch_bounds__(rows_threads(LOGS), rows_min_waves(LOGS)) void k_rows(
    KParams<A> P, const TIn *__restrict__ a, const TIn *__restrict__ b, TOut *__restrict__ c,
    size_t units) {
  using W = typename A::word;
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int N = Gr::N, TP = N / 16, PB = rows_threads(LOGS) / TP, G = Gr::G, NP = Gr::NP;
  constexpr bool kNT = NTTMUL_NT && (L1 == 0 || NTTMUL_NT_MP);
  __shared__ W lds[PB][lds_regions<W>()][NP];

  const int pb = threadIdx.x / TP, j = threadIdx.x % TP;
  const size_t u = (size_t)blockIdx.x * PB + pb;
  const bool live = u < units;
  const int row = L1 ? (int)(u & ((1u << L1) - 1)) : 0;
  // (the square split's intermediates are tiled, c8_tile: row u = (p, m) keeps its element e at
  // p 2^16 + (e >> 4) 2^12 + 16 m + (e & 15), i.e. register k of lane j at 4096 k + 16 m + j)
  constexpr bool kTile = c8_tile(LOGS, L1);
  constexpr int kRS = kTile ? 256 : 1;  // word stride of Gr::off(0, k)
  const size_t base_g = kTile ? ((u >> 8) << 16) + ((u & 255) << 4) + Gr::base(0, j)
                              : u * N + Gr::base(0, j);
  // threads past the batch end read unit 0 (always valid) instead of branching per load; their
  // results are never stored
  const size_t base_l = live ? base_g : (size_t)Gr::base(0, j);
  const size_t base_r = NTTMUL_HOOK_ROWS_LD(base_l, u, N, Gr::base(0, j));

  // NTTMUL_C5_BUF, the square split's row pass: one descriptor per polynomial (its 16 rows per
  // block share it), 32-bit lane offsets, each register's constant offset in the scalar offset
  constexpr bool kRowBuf = kTile && NTTMUL_C5_BUF && !NTTMUL_ROWS_HOOKED && sizeof(W) == 8 &&
                           sizeof(TIn) == 8 && sizeof(TOut) == 8 && !kNT;
  const size_t rpoly = (((size_t)blockIdx.x * PB) >> 8) << 16;  // block-uniform
  const int rlane = (int)(((u & 255) << 4) + Gr::base(0, j));
  CLK_STAMP(0);
  if constexpr (PRIO) NTTMUL_HOOK_PRIO0(u);  // rows_prio
  W x[16], y[16];
  // NTTMUL_CPOL >= 0: a, b, c of a one-product-per-block u32 product through buffer loads /
  // stores (descriptor from block-uniform values, 32-bit per-lane offsets, nt by default)
  // (64-bit words of the square split take kRowBuf below: one descriptor per polynomial and the
  // constant offsets in the scalar offset; round 2's form, an offset per register, measured
  // +0.8 % at C5 with its row pass at 131 VGPRs instead of 126)
  constexpr bool kCpol = NTTMUL_CPOL >= 0 && PB == 1 && L1 == 0 && sizeof(W) == 4 &&
                         sizeof(TIn) == 4 && sizeof(TOut) == 4;
  constexpr int kAux = NTTMUL_CPOL < 0 ? 0 : NTTMUL_CPOL;
  constexpr int kAuxSt = NTTMUL_CPOL_ST < 0 ? 0 : NTTMUL_CPOL_ST;
  // n = 1024 one-wave products (C2: a single generation of waves that all wait for their loads):
  // a's forward transform runs while b is still landing (NTTMUL_SPLIT_AB)
  constexpr bool kSplitAB = NTTMUL_SPLIT_AB && kCpol && LOGS == 10;
  if constexpr (kCpol) {
    const size_t ub = live ? (size_t)blockIdx.x : 0;
    const auto ra = span_rsrc(a + ub * N, N), rb = span_rsrc(b + ub * N, N);
    if constexpr (kSplitAB) {  // all of a first: a's transform starts before b has landed
#pragma unroll
      for (int k = 0; k < 16; k++) x[k] = (W)buf_ld32<kAux>(ra, (Gr::base(0, j) + Gr::off(0, k)) * 4);
#pragma unroll
      for (int k = 0; k < 16; k++) y[k] = (W)buf_ld32<kAux>(rb, (Gr::base(0, j) + Gr::off(0, k)) * 4);
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++) {
        if constexpr (NTTMUL_BUF_SOFF) {
          const int vo = Gr::base(0, j) * 4, so = Gr::off(0, k) * 4;
          x[k] = (W)buf_ld32<kAux>(ra, vo, so);
          y[k] = (W)buf_ld32<kAux>(rb, vo, so);
        } else {
          const int off = (Gr::base(0, j) + Gr::off(0, k)) * 4;
          x[k] = (W)buf_ld32<kAux>(ra, off);
          y[k] = (W)buf_ld32<kAux>(rb, off);
        }
      }
    }
  } else if constexpr (kRowBuf) {
    // (units is a multiple of 256 rows here, so every row of the block is live)
    const auto ra = span_rsrc(a + rpoly, 65536), rb = span_rsrc(b + rpoly, 65536);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int so = Gr::off(0, k) * kRS * 8;
      x[k] = (W)buf_ld64<0>(ra, rlane * 8, so);
      y[k] = (W)buf_ld64<0>(rb, rlane * 8, so);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++) {
      x[k] = to_word<W>(ld_stream<kNT>(a + base_r + Gr::off(0, k) * kRS));
      y[k] = to_word<W>(ld_stream<kNT>(b + base_r + Gr::off(0, k) * kRS));
    }
  }
  NTTMUL_HOOK_ROWS_INPUT(x, y, u, j);
  W *lx = lds[pb][0], *ly = lds[pb][lds_regions<W>() - 1];
  constexpr int D = NTTMUL_BASE_D ? A::kBaseD : 0;
  TwPair<W> zw[16];
  if constexpr (kSplitAB) {  // a's forward transform, then b's (each waits only for its loads)
    fwd_all<A, LOGS, 0, 1, D>(P.ar, x, y, lx, ly, P.fw, j, row, L1, zw);
    fwd_all<A, LOGS, 0, 1, D>(P.ar, y, x, lx, ly, P.fw, j, row, L1, zw);
  } else {
    fwd_all<A, LOGS, 0, 2, D>(P.ar, x, y, lx, ly, P.fw, j, row, L1, zw);
  }
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
  base_mult<A, LOGS, D>(P.ar, x, y, zw, j);
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  inv_all<A, LOGS, G - 1, L1 == 0, D>(P, x, y, lx, ly, P.iw, j, row, L1);
  NTTMUL_HOOK_ROWS_OUTPUT(x, c, base_g, live);
  if constexpr (kCpol) {
    if (live) {
      const auto rc = span_rsrc(c + (size_t)blockIdx.x * N, N);
#pragma unroll
      for (int k = 0; k < 16; k++) {
        W v = x[k];
        if (!A::kInvCanonical) v = P.ar.canon_inv(v);
        if constexpr (NTTMUL_BUF_SOFF)
          buf_st32<kAuxSt>(rc, Gr::base(0, j) * 4, (uint32_t)v, Gr::off(0, k) * 4);
        else
          buf_st32<kAuxSt>(rc, (Gr::base(0, j) + Gr::off(0, k)) * 4, (uint32_t)v);
      }
    }
    CLK_STAMP(1);
    return;
  }
  if constexpr (kRowBuf) {
    const auto rc = span_rsrc(c + rpoly, 65536);
#pragma unroll
    for (int k = 0; k < 16; k++) buf_st64<0>(rc, rlane * 8, (uint64_t)x[k], Gr::off(0, k) * kRS * 8);
    CLK_STAMP(1);
    return;
  }
  if (live) {
    const size_t base_w = NTTMUL_HOOK_ROWS_ST(base_g, u, N, Gr::base(0, j));
#pragma unroll
    for (int k = 0; k < 16; k++) {
      W v = x[k];
      if (L1 == 0 && !A::kInvCanonical) v = P.ar.canon_inv(v);
      st_stream<kNT>(c + base_w + Gr::off(0, k) * kRS, (TOut)v);
    }
  }
  CLK_STAMP(1);
}

// s_sleep argument between the device server's polls (x 64 cycles: 2 = 53 ns at 2.4 GHz)
#ifndef NTTMUL_SERVER_POLL_SLEEP
#define NTTMUL_SERVER_POLL_SLEEP 2
#endif
// The wide single-product path of the device server (n = 256, one product: every call of the
// reference's ntt256_product4 / product1 shims).  The one-wave path gives a product 16 lanes of
// 16 coefficients (a and b on two lane groups, the inverse on one), so a call is about 1,100
// dependent VALU instructions on one SIMD; here each polynomial is a whole wave of 4
// coefficients per lane: wave 0 transforms a while wave 1 transforms b, and wave 0 runs the base
// multiplication and the inverse, about 3x fewer instructions on the critical path for 7 LDS
// exchanges instead of 2.  Register groups of two stages: layout P holds element bits P, P + 1 in
// the four registers, e = (t mod 2^P) | (t >> P) << (P + 2) | i << P for lane t, register i.
// Types as in the fused product (Arith32P, NTTMUL_P_TYPED 2), with the planner's twiddle table
// re-typed per entry in LDS (fu: every pair unsigned, fs: every pair signed) because the group
// boundaries differ: the second stage of a group multiplies the first stage's differences as
// signed values with signed pairs (odd entries), the first reads unsigned lazy values, and the
// last forward stage leaves its differences signed for the base multiplication.
template <int P_>
__device__ __forceinline__ int wl_elem(int t, int i) {
  return (t & ((1 << P_) - 1)) | ((t >> P_) << (P_ + 2)) | (i << P_);
}
__device__ __forceinline__ int wl_pad(int e) { return e + (e >> 5); }
// one wave's four registers from layout PF to layout PT through its LDS region
template <int PF, int PT>
__device__ __forceinline__ void wl_exchange(uint32_t (&x)[4], uint32_t *lx, int t) {
#pragma unroll
  for (int i = 0; i < 4; i++) lx[wl_pad(wl_elem<PF>(t, i))] = x[i];
  xsync<1>();
#pragma unroll
  for (int i = 0; i < 4; i++) x[i] = lx[wl_pad(wl_elem<PT>(t, i))];
  xsync<1>();
}
// A lane's twiddle pairs for one request (the same every request: loaded into registers once,
// so the transforms read no memory): forward f[0..8] in stage order, the base block's z, inverse
// i[0..7] in stage order (5, 4, 3, 2, 1)
struct WideTw {
  TwPair<uint32_t> f[9], z, i[8];
};
__device__ __forceinline__ WideTw wide_tw(const TwPair<uint32_t> *fu, const TwPair<uint32_t> *fs,
                                          const TwPair<uint32_t> *iw, int t) {
  WideTw w;
  const int k3 = 8 + ((t >> 4) << 1), k5 = 32 + ((t >> 2) << 1);
  w.f[0] = fu[1];               // stage 0: entry 1
  w.f[1] = fu[2];               // stage 1: entries 2 (sums) and 3 (differences)
  w.f[2] = fs[3];
  w.f[3] = fu[4 + (t >> 4)];    // stage 2: entry 4 + e >> 6 (layout 4)
  w.f[4] = fu[k3];              // stage 3: entry 8 + e >> 5
  w.f[5] = fs[k3 + 1];
  w.f[6] = fu[16 + (t >> 2)];   // stage 4: entry 16 + e >> 4 (layout 2)
  w.f[7] = fu[k5];              // stage 5: entry 32 + e >> 3
  w.f[8] = fs[k5 + 1];
  w.z = fs[32 + (t >> 1)];      // block lane t: elements 4t .. 4t + 3 (layout 0)
  w.i[0] = iw[k5];
  w.i[1] = iw[k5 + 1];
  w.i[2] = iw[16 + (t >> 2)];
  w.i[3] = iw[k3];
  w.i[4] = iw[k3 + 1];
  w.i[5] = iw[4 + (t >> 4)];
  w.i[6] = iw[2];
  w.i[7] = iw[3];
  return w;
}
// Layout changes inside the wave without LDS.  Layouts 6 and 4 differ by swapping register bit 0
// with lane bit 4 and register bit 1 with lane bit 5: one v_permlane16_swap / v_permlane32_swap
// per register pair.  Layouts 4 and 2 differ by register bits 0, 1 against lane bits 2, 3: two
// DPP row shifts (by 4 or 8 lanes within a 16-lane row) and two selects per register pair.  Both
// are involutions, so the inverse uses them back.
__device__ __forceinline__ void wl_swap_64(uint32_t (&x)[4]) {
  auto s0 = __builtin_amdgcn_permlane16_swap(x[0], x[1], false, false);
  auto s1 = __builtin_amdgcn_permlane16_swap(x[2], x[3], false, false);
  x[0] = s0[0], x[1] = s0[1], x[2] = s1[0], x[3] = s1[1];
  auto s2 = __builtin_amdgcn_permlane32_swap(x[0], x[2], false, false);
  auto s3 = __builtin_amdgcn_permlane32_swap(x[1], x[3], false, false);
  x[0] = s2[0], x[2] = s2[1], x[1] = s3[0], x[3] = s3[1];
}
// register bit r <-> lane bit log2(SH) for the pair (x[A], x[A + 1 << r]): lanes with that bit
// set take the partner register's value from SH lanes below, the others from SH lanes above
template <int SH, int A, int B>
__device__ __forceinline__ void wl_swap_dpp(uint32_t (&x)[4], int t) {
  const uint32_t up = __builtin_amdgcn_update_dpp(0u, x[B], 0x110 + SH, 0xF, 0xF, false);  // row_shr
  const uint32_t dn = __builtin_amdgcn_update_dpp(0u, x[A], 0x100 + SH, 0xF, 0xF, false);  // row_shl
  const bool hi = (t & SH) != 0;
  x[A] = hi ? up : x[A];
  x[B] = hi ? x[B] : dn;
}
__device__ __forceinline__ void wl_swap_42(uint32_t (&x)[4], int t) {
  wl_swap_dpp<4, 0, 1>(x, t);
  wl_swap_dpp<4, 2, 3>(x, t);
  wl_swap_dpp<8, 0, 2>(x, t);
  wl_swap_dpp<8, 1, 3>(x, t);
}
// forward CT, stages 0-5 of the incomplete transform (D = 2), X canonical on entry (the API
// contract); layout 6 in, layout 2 out (element bits 2, 3 in the registers)
__device__ __forceinline__ void wide_fwd(const Arith32P &ar, uint32_t (&x)[4], const WideTw &w,
                                         uint32_t *lx, int t) {
  // stage 0 (d 128: register bit 1)
  ar.template ct<true, false, true>(x[0], x[2], w.f[0].w, w.f[0].ws);
  ar.template ct<true, false, true>(x[1], x[3], w.f[0].w, w.f[0].ws);
  // stage 1 (d 64: register bit 0), the second pair on stage 0's differences
  ar.template ct<false, false, false>(x[0], x[1], w.f[1].w, w.f[1].ws);
  ar.template ct<false, true, false>(x[2], x[3], w.f[2].w, w.f[2].ws);
  wl_swap_64(x);
  // stage 2 (d 32: register bit 1)
  ar.template ct<false, false, true>(x[0], x[2], w.f[3].w, w.f[3].ws);
  ar.template ct<false, false, true>(x[1], x[3], w.f[3].w, w.f[3].ws);
  // stage 3 (d 16: register bit 0)
  ar.template ct<false, false, false>(x[0], x[1], w.f[4].w, w.f[4].ws);
  ar.template ct<false, true, false>(x[2], x[3], w.f[5].w, w.f[5].ws);
  wl_swap_42(x, t);
  // stage 4 (d 8: register bit 1)
  ar.template ct<false, false, true>(x[0], x[2], w.f[6].w, w.f[6].ws);
  ar.template ct<false, false, true>(x[1], x[3], w.f[6].w, w.f[6].ws);
  // stage 5 (d 4: register bit 0); the differences stay signed for the base multiplication
  ar.template ct<false, false, true>(x[0], x[1], w.f[7].w, w.f[7].ws);
  ar.template ct<false, true, true>(x[2], x[3], w.f[8].w, w.f[8].ws);
}
// inverse GS from layout 2 (the first D = 2 stages are the base multiplication's), F folded into
// stage 0; leaves layout 6 (e = t + 64 i), canonical
__device__ __forceinline__ void wide_inv(const KParams<Arith32P> &P, uint32_t (&x)[4],
                                         const WideTw &w, uint32_t *lx, int t) {
  P.ar.gs(x[0], x[1], w.i[0].w, w.i[0].ws);  // stage 5 (register bit 0)
  P.ar.gs(x[2], x[3], w.i[1].w, w.i[1].ws);
  P.ar.gs(x[0], x[2], w.i[2].w, w.i[2].ws);  // stage 4 (register bit 1)
  P.ar.gs(x[1], x[3], w.i[2].w, w.i[2].ws);
  wl_swap_42(x, t);
  P.ar.gs(x[0], x[1], w.i[3].w, w.i[3].ws);  // stage 3
  P.ar.gs(x[2], x[3], w.i[4].w, w.i[4].ws);
  P.ar.gs(x[0], x[2], w.i[5].w, w.i[5].ws);  // stage 2
  P.ar.gs(x[1], x[3], w.i[5].w, w.i[5].ws);
  wl_swap_64(x);
  P.ar.gs(x[0], x[1], w.i[6].w, w.i[6].ws);  // stage 1
  P.ar.gs(x[2], x[3], w.i[7].w, w.i[7].ws);
  P.ar.gs_scaled(x[0], x[2], P.f, P.fs, P.wf, P.wfs);  // stage 0 with F
  P.ar.gs_scaled(x[1], x[3], P.f, P.fs, P.wf, P.wfs);
}

// Small-transaction device server (host calls of at most 1024 words per operand, e.g. the
// reference's ntt256_product4 through the compat shims; nttmul.cpp Server).  Wave 0 polls the
// request's go word (sequence number << 8 | product count) with system-scope reads; on a new word
// it takes the request (system acquire), pulls a and b in system-scope loads, runs the product on
// twiddles copied into LDS at entry (no L2 / HBM latency inside the transforms) and writes c back
// in system-scope write-through stores (the host takes the request as done when every word of c
// has changed from the pending marker).  The request half of the mailbox (req) is device memory
// the host writes through its BAR mapping, so polls and operand loads stay on the device; c goes
// to host memory (launch.hpp ServerReq / ServerBox).  n = 256: the two-wave path above, one pair
// of waves per product of the request (up to 4); n = 1024: a and b transformed on two waves.  Otherwise one wave runs the fused product
// of k_rows (64 / (n / 16) products per wave,
// exchanges ordered per wave; a single product of n = 512 transforms a and b on two lane groups,
// b's result handed to a's lanes by lane permutes).  It leaves on stop, after idle_ticks without
// a request or after life_ticks in all (the host relaunches it on demand), so every wave always
// ends -- the FPGA's GO / done-all handshake without a kernel launch per call.
template <class A, int LOGS>
__global__ __launch_bounds__(LOGS == 8 ? 512 : LOGS == 9 ? 64 : 128) void k_server(
    KParams<A> P, const ServerReq *req, ServerBox *box, unsigned tw_pairs,
    unsigned long long idle_ticks, unsigned long long life_ticks) {
  using W = typename A::word;
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int N = Gr::N, TP = N / 16, PB = 64 / TP, G = Gr::G, NP = Gr::NP;
  static_assert(sizeof(W) == 4 && TP <= 64, "u32 words, n <= 1024");
  constexpr bool kWide = LOGS == 8 && IsPlantard<A>::value && NTTMUL_BASE_D && A::kBaseD == 2;
  constexpr bool kPair = LOGS == 10;  // n = 1024 (one product per request): a and b on two waves
  constexpr int KW = ServerBox::kWords, NT = LOGS == 8 ? 512 : LOGS == 9 ? 64 : 128;
  __shared__ W lds[kWide ? 2 * PB : PB < 2 ? 2 : PB][NP];
  __shared__ uint4 stg[2][KW / 4];  // a, b as loaded (c as stored reuses stg[0])
  __shared__ TwPair<W> twf[N], twi[N];  // launch_server: tw_pairs <= n
  __shared__ TwPair<W> wfu[kWide ? N : 1], wfs[kWide ? N : 1];
  __shared__ unsigned s_go, s_quit;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, pb = lane / TP, j = lane % TP;
  for (unsigned i = threadIdx.x; i < tw_pairs; i += NT) {
    const TwPair<W> f = P.fw[i];
    twf[i] = f;
    twi[i] = P.iw[i];
    if constexpr (kWide) {  // the planner's per-entry form (arith_select.hpp p_signed_fw_entry)
      const W sg = f.w >> 31;
      const bool s = p_signed_fw_entry(LOGS, i);
      wfu[i] = {f.w, s ? f.ws - sg : f.ws};
      wfs[i] = {f.w, s ? f.ws : f.ws + sg};
    }
  }
  P.fw = twf;
  P.iw = twi;
  W *lx = lds[pb];
  constexpr int D = NTTMUL_BASE_D ? A::kBaseD : 0;
  unsigned seen = __hip_atomic_load(&box->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  seen = __builtin_amdgcn_readfirstlane(seen);
  __syncthreads();  // the twiddles in LDS before the first transform
  WideTw wtw;
  if constexpr (kWide) wtw = wide_tw(wfu, wfs, twi, lane);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long last = t0;
  // one poll at a time, NTTMUL_SERVER_POLL_SLEEP apart.  (Rounds 4b-4f kept three polls in
  // flight 16 x 64 cycles apart, sized for reads across PCIe; with the request in device memory a
  // single poll is 1 us faster per request, and with it in host memory too:
  // tools/microbench/mailbox_latency.hip, profiles/r4/mailbox/)
  constexpr int kSleep = NTTMUL_SERVER_POLL_SLEEP;
  for (;;) {
    unsigned go = seen;
    bool quit = false;
    if (wave == 0) {
      for (;;) {
        go = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&req->go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        if (go != seen) break;
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        if ((quit = now - last > idle_ticks || now - t0 > life_ticks)) break;
        __builtin_amdgcn_s_sleep(kSleep);
      }
    }
    if constexpr (NT > 64) {  // the other wave waits at the barrier while wave 0 polls
      if (threadIdx.x == 0) s_go = go, s_quit = quit;
      __syncthreads();
      go = __builtin_amdgcn_readfirstlane(s_go);
      quit = __builtin_amdgcn_readfirstlane(s_quit) != 0;
    }
    if (quit) break;
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    const int count = (int)(go & 0xFFu);
    if (count == (int)ServerBox::kStop || count > PB) break;  // stop (count > PB: never posted)
    // the host's a, b before go (only the waves that load them: on the n = 256 path eight waves
    // invalidating at once cost a single product 0.5 us)
    if (!kWide || (wave >> 1) < count) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
#ifdef NTTMUL_CLOCK_STAMPS
    unsigned long long st[6];
    st[0] = __builtin_amdgcn_s_memrealtime();
#endif
    const int q4 = count * (N / 4);  // 16-byte quads per operand (count <= PB, so <= KW / 4)
    if (kWide) {
      if constexpr (kWide) {
        // product p = wave / 2 of the request (count <= 4): wave 2p loads and transforms a_p,
        // wave 2p + 1 b_p (layout 6, system-scope loads: the host's writes reach memory behind
        // any cached copy); waves of products past count only keep the barriers
        const int prod = wave >> 1, opnd = wave & 1;
        const bool mine = prod < count;
        uint32_t x[4];
        uint32_t *lw = lds[wave];
        if (mine) {
          const auto ro = span_rsrc((opnd ? req->b : req->a) + prod * N, N);
#pragma unroll
          for (int i = 0; i < 4; i++)
            x[i] = __builtin_amdgcn_raw_buffer_load_b32(ro, (lane + 64 * i) * 4, 0, 17);
#ifdef NTTMUL_CLOCK_STAMPS
          __builtin_amdgcn_s_waitcnt(0);
          st[1] = __builtin_amdgcn_s_memrealtime();
          st[4] = __builtin_amdgcn_s_memtime();
#endif
          wide_fwd(P.ar, x, wtw, lw, lane);
          // both transforms to the block layout (one 4-coefficient base block per lane)
#pragma unroll
          for (int i = 0; i < 4; i++) lw[wl_pad(wl_elem<2>(lane, i))] = x[i];
        }
        __syncthreads();
        if (mine && opnd == 0) {
          uint32_t y[4];
#pragma unroll
          for (int i = 0; i < 4; i++) {
            x[i] = lds[wave][wl_pad(wl_elem<0>(lane, i))];
            y[i] = lds[wave + 1][wl_pad(wl_elem<0>(lane, i))];
          }
          xsync<1>();
          // block lane: elements 4 lane .. 4 lane + 3, a residue mod x^4 -+ w with w the stage-5
          // entry 32 + lane / 2, minus for odd lanes (the stage's differences)
          P.ar.basemul4_lane(x, y, wtw.z.w, wtw.z.ws, lane & 1);
          wl_exchange<0, 2>(x, lw, lane);
          wide_inv(P, x, wtw, lw, lane);
#ifdef NTTMUL_CLOCK_STAMPS
          __builtin_amdgcn_sched_barrier(0);
          st[2] = __builtin_amdgcn_s_memrealtime();
          st[5] = __builtin_amdgcn_s_memtime();
#endif
          // (the host watches c itself, see below: system-scope write-through stores)
          const auto rc = span_rsrc(box->c + prod * N, N);
#pragma unroll
          for (int i = 0; i < 4; i++)
            __builtin_amdgcn_raw_buffer_store_b32(x[i], rc, (lane + 64 * i) * 4, 0, 17);
        }
      }
    } else if (kPair) {
      if constexpr (kPair) {
        // n = 1024: wave w loads operand w (system scope, through stg[w]) and runs the fused
        // kernel's forward groups on it in its own LDS region -- the one-wave path transforms a
        // and b on the same lanes, twice the instructions on one SIMD; wave 1 hands b's
        // transform to wave 0's registers through LDS (same layout), and wave 0 runs the base
        // multiplication and the inverse
        {
          const auto ro = span_rsrc(wave ? req->b : req->a, KW);
          for (int i = lane; i < N / 4; i += 64) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(ro, i * 16, 0, 17);
            stg[wave][i] = make_uint4(v[0], v[1], v[2], v[3]);
          }
        }
        xsync<1>();
        W x[16], y[16];
        {
          const W *src = (const W *)stg[wave];
#pragma unroll
          for (int k = 0; k < 16; k++) x[k] = src[Gr::base(0, j) + Gr::off(0, k)];
        }
#ifdef NTTMUL_CLOCK_STAMPS
        st[1] = __builtin_amdgcn_s_memrealtime();
        st[4] = __builtin_amdgcn_s_memtime();
#endif
        TwPair<W> zw[16];
        W *lw = lds[wave];
        fwd_all<A, LOGS, 0, 1, D, 1>(P.ar, x, y, lw, lw, P.fw, j, 0, 0, zw);
        W *hand = (W *)stg[1];  // (b's input, already in wave 1's registers)
        if (wave == 1) {
#pragma unroll
          for (int k = 0; k < 16; k++) hand[k * 64 + lane] = x[k];
        }
        __syncthreads();
        if (wave == 0) {
#pragma unroll
          for (int k = 0; k < 16; k++) y[k] = hand[k * 64 + lane];
          base_mult<A, LOGS, D>(P.ar, x, y, zw, j);
          inv_all<A, LOGS, G - 1, true, D, 1>(P, x, y, lw, lw, P.iw, j, 0, 0);
#ifdef NTTMUL_CLOCK_STAMPS
          __builtin_amdgcn_sched_barrier(0);
          st[2] = __builtin_amdgcn_s_memrealtime();
          st[5] = __builtin_amdgcn_s_memtime();
#endif
          W *sc = (W *)stg[0];
#pragma unroll
          for (int k = 0; k < 16; k++) {
            W v = x[k];
            if (!A::kInvCanonical) v = P.ar.canon_inv(v);
            sc[Gr::base(0, j) + Gr::off(0, k)] = v;
          }
          xsync<1>();
          const auto rc = span_rsrc(box->c, KW);  // (system-scope write-through, see below)
          for (int i = lane; i < N / 4; i += 64) {
            const uint4 v = stg[0][i];
            __attribute__((ext_vector_type(4))) uint32_t w = {v.x, v.y, v.z, v.w};
            __builtin_amdgcn_raw_buffer_store_b128(w, rc, i * 16, 0, 17);
          }
        }
      }
    } else if (wave == 0) {
      {  // system-scope (sc0 sc1) loads: the host's writes reach memory behind any cached copy
        const auto ra = span_rsrc(req->a, KW), rb = span_rsrc(req->b, KW);
        for (int i = lane; i < q4; i += 64) {
          const auto va = __builtin_amdgcn_raw_buffer_load_b128(ra, i * 16, 0, 17);
          const auto vb = __builtin_amdgcn_raw_buffer_load_b128(rb, i * 16, 0, 17);
          stg[0][i] = make_uint4(va[0], va[1], va[2], va[3]);
          stg[1][i] = make_uint4(vb[0], vb[1], vb[2], vb[3]);
        }
      }
      xsync<1>();
      const W *sa = (const W *)stg[0], *sb = (const W *)stg[1];
      // one product of n <= 512: lane group 0 transforms a, group 1 b (then hands b over)
      const bool split = PB >= 2 && count == 1;
      const bool live = pb < count;
      W x[16], y[16];
      {
        const int base = (live ? pb : 0) * N + Gr::base(0, j);
        const W *src = split && pb == 1 ? sb : sa;
#pragma unroll
        for (int k = 0; k < 16; k++) {
          x[k] = src[base + Gr::off(0, k)];
          y[k] = sb[base + Gr::off(0, k)];
        }
      }
      TwPair<W> zw[16];
#ifdef NTTMUL_CLOCK_STAMPS
      st[1] = __builtin_amdgcn_s_memrealtime();
      st[4] = __builtin_amdgcn_s_memtime();
#endif
      if (split) {
        fwd_all<A, LOGS, 0, 1, D, 1>(P.ar, x, y, lx, lx, P.fw, j, 0, 0, zw);
#pragma unroll
        for (int k = 0; k < 16; k++)  // group 1's transformed b to group 0's lanes, same j
          y[k] = (W)__builtin_amdgcn_ds_bpermute((lane + TP) << 2, (int)x[k]);
      } else {
        fwd_all<A, LOGS, 0, 2, D, 1>(P.ar, x, y, lx, lx, P.fw, j, 0, 0, zw);
      }
      base_mult<A, LOGS, D>(P.ar, x, y, zw, j);
      inv_all<A, LOGS, G - 1, true, D, 1>(P, x, y, lx, lx, P.iw, j, 0, 0);
#ifdef NTTMUL_CLOCK_STAMPS
      __builtin_amdgcn_sched_barrier(0);
      st[2] = __builtin_amdgcn_s_memrealtime();
      st[5] = __builtin_amdgcn_s_memtime();
#endif
      W *sc = (W *)stg[0];
      if (live) {
        const int base = pb * N + Gr::base(0, j);
#pragma unroll
        for (int k = 0; k < 16; k++) {
          W v = x[k];
          if (!A::kInvCanonical) v = P.ar.canon_inv(v);
          sc[base + Gr::off(0, k)] = v;
        }
      }
      xsync<1>();
      // (the host watches c itself: a word that is no longer ServerBox::kPending has landed, so
      // no release fence or done word is needed before polling again.  The stores are
      // system-scope write-through (sc0 sc1): plain stores to the host-coherent mailbox stay in
      // the L2 until a release or the kernel's end -- measured: 20 ms per request, the idle exit)
      const auto rc = span_rsrc(box->c, KW);
      for (int i = lane; i < q4; i += 64) {
        const uint4 v = stg[0][i];
        __attribute__((ext_vector_type(4))) uint32_t w = {v.x, v.y, v.z, v.w};
        __builtin_amdgcn_raw_buffer_store_b128(w, rc, i * 16, 0, 17);  // aux 17: sc0 sc1
      }
    }
#ifdef NTTMUL_CLOCK_STAMPS  // diagnostic build: c landed (fence), then the stamps, then done
    if (wave == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st[3] = __builtin_amdgcn_s_memrealtime();
      if (threadIdx.x == 0)  // vector stores from lane 0, released with done below
        for (int k = 0; k < 6; k++) box->stamp[k] = st[k];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&box->done, go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#endif
    seen = go;
    last = now;
    // the next request's loads land in stg / lds after every lane has stored c
    if constexpr (NT > 64) __syncthreads(); else xsync<1>();
  }
}

// Standalone transforms, one polynomial per unit of 2^LOGS coefficients.
//   DIR 0 (forward): NTT/ntt.C:342-371 mulntt_ct_std2rev — standard order in, bit-reversed out;
//     with L1 > 0 this is the row pass after k_cols_fwd.  Output canonical when L1 == 0 or
//     the row pass is the last forward step (always, for the forward direction).
//   DIR 1 (inverse): NTT/ntt.C:428-451 nttmul_gs_rev2std followed by the n^-1 scaling of
//     ntt256.C:12 (P.f = n^-1 here), so inverse(forward(a)) == a; with L1 > 0 this is the row
//     pass before k_cols_inv and the output stays lazy.
// Transforms of 32-bit words with L1 == 0 take two polynomials per thread group (the product
// kernel's a and b form: one twiddle load and one exchange barrier per stage serve both, and
// twice the independent butterflies per lane).
template <class A, int L1, int DIR>
constexpr int xform_upg() { return L1 == 0 && sizeof(typename A::word) == 4 ? 2 : 1; }
template <class A, class TIn, class TOut, int LOGS, int L1, int DIR>
__global__ __launch_bounds__(256) void k_xform(KParams<A> P, const TIn *__restrict__ in,
                                               TOut *__restrict__ out, size_t units) {
  using W = typename A::word;
  using Gr = Groups<LOGS, kWT<A, LOGS>()>;
  constexpr int N = Gr::N, TP = N / 16, PB = 256 / TP, G = Gr::G, NP = Gr::NP;
  constexpr int GIN = DIR == 0 ? 0 : G - 1, GOUT = DIR == 0 ? G - 1 : 0;
  constexpr int UPG = xform_upg<A, L1, DIR>();
  __shared__ W lds[PB][UPG][NP];
  const int pb = threadIdx.x / TP, j = threadIdx.x % TP;
  const size_t u = ((size_t)blockIdx.x * PB + pb) * UPG;
  const bool live = u < units, live2 = UPG == 2 && u + 1 < units;
  const int row = L1 ? (int)(u & ((1u << L1) - 1)) : 0;
  // the square split's tiled intermediate (c8_tile, as k_rows): the forward row pass reads it,
  // the inverse row pass writes it
  constexpr bool kTile = c8_tile(LOGS, L1);
  constexpr int kRS = kTile ? 256 : 1;
  static_assert(!kTile || UPG == 1, "one polynomial per thread group on the tiled layout");
  const auto tbase = [&](size_t v, int g) {
    return kTile ? ((v >> 8) << 16) + ((v & 255) << 4) + Gr::base(g, j) : v * N + Gr::base(g, j);
  };
  const size_t base_in = DIR == 0 ? tbase(live ? u : 0, GIN) : (live ? u : 0) * N + Gr::base(GIN, j);
  const size_t base_in2 = (live2 ? u + 1 : live ? u : 0) * N + Gr::base(GIN, j);
  constexpr int kRSI = DIR == 0 ? kRS : 1, kRSO = DIR == 1 ? kRS : 1;
  W x[16], y[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    x[k] = to_word<W>(in[base_in + Gr::off(GIN, k) * kRSI]);
    if (UPG == 2) y[k] = to_word<W>(in[base_in2 + Gr::off(GIN, k)]);
  }
  TwPair<W> zw[16];
  if (DIR == 0)
    fwd_all<A, LOGS, 0, UPG>(P.ar, x, y, lds[pb][0], lds[pb][UPG - 1], P.fw, j, row, L1, zw);
  else
    inv_all<A, LOGS, G - 1, L1 == 0, 0, 0, UPG>(P, x, y, lds[pb][0], lds[pb][UPG - 1], P.iw, j, row, L1);
  if (live) {
    const size_t base_out = DIR == 1 ? tbase(u, GOUT) : u * N + Gr::base(GOUT, j);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      W v = x[k];
      if (DIR == 0)
        v = P.ar.canon(v);
      else if (L1 == 0 && !A::kInvCanonical)
        v = P.ar.canon_inv(v);
      out[base_out + Gr::off(GOUT, k) * kRSO] = (TOut)v;
    }
  }
  if (live2) {
    const size_t base_out = (u + 1) * N + Gr::base(GOUT, j);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      W v = y[k];
      if (DIR == 0)
        v = P.ar.canon(v);
      else if (!A::kInvCanonical)
        v = P.ar.canon_inv(v);
      out[base_out + Gr::off(GOUT, k)] = (TOut)v;
    }
  }
}

// c = a * b mod q coefficient-wise (NTT/ntt.C:131-137 mul_array), canonical in and out:
// two Montgomery products, the second by R^2 mod q (P.f holds R^2 mod q for this kernel).
template <class A, class IO>
__global__ __launch_bounds__(256) void k_pointwise(KParams<A> P, const IO *__restrict__ a,
                                                   const IO *__restrict__ b, IO *__restrict__ c,
                                                   size_t total) {
  using W = typename A::word;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const W t = P.ar.mont((W)a[i], (W)b[i]);
  c[i] = (IO)P.ar.canon_inv(P.ar.mont(t, P.f));  // mont: [0, 2q)
}

// Column pass, forward: global stages 0..L1-1 of CT on a and b.  Thread = one column
// (e = col + m * 2^LOGS, m < 2^L1); lanes on consecutive columns -> coalesced rows.
template <class A, class TIn, int L1, int NPOLY = 2>
__global__ __launch_bounds__(256) void k_cols_fwd(KParams<A> P, const TIn *__restrict__ a,
                                                  const TIn *__restrict__ b,
                                                  typename A::word *__restrict__ ta,
                                                  typename A::word *__restrict__ tb, size_t batch,
                                                  int logs) {
  using W = typename A::word;
  constexpr int M = 1 << L1;
  const size_t ncol = (size_t)1 << logs;
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= batch * ncol) return;
  const size_t p = gid >> logs, col = gid & (ncol - 1);
  const size_t base = (p << (logs + L1)) + col;
  const size_t base_r = NTTMUL_HOOK_COLS_LD(base, p, logs + L1, col, 0);
  const size_t base_w = NTTMUL_HOOK_COLS_ST(base, p, logs + L1, col);
  W x[M], y[M];
#pragma clang loop unroll(full)
  for (int m = 0; m < M; m++) {
    x[m] = (W)ld_stream<NTTMUL_NT_COLS>(a + base_r + ((size_t)m << logs));
    y[m] = NPOLY == 2 ? (W)ld_stream<NTTMUL_NT_COLS>(b + base_r + ((size_t)m << logs)) : W(0);
  }
#pragma clang loop unroll(full)
  for (int st = 0; st < L1; st++) {
    const int dist = M >> (st + 1);
#pragma clang loop unroll(full)
    for (int m = 0; m < M; m++) {
      if (m & dist) continue;
      const TwPair<W> t = P.fw[(1 << st) + (m >> (L1 - st))];
      P.ar.ct(x[m], x[m + dist], t.w, t.ws);
      if (NPOLY == 2) P.ar.ct(y[m], y[m + dist], t.w, t.ws);
    }
  }
#pragma clang loop unroll(full)
  for (int m = 0; m < M; m++) {
    st_stream<NTTMUL_NT_COLS>(ta + base_w + ((size_t)m << logs), x[m]);
    if (NPOLY == 2) st_stream<NTTMUL_NT_COLS>(tb + base_w + ((size_t)m << logs), y[m]);
  }
}

// Column pass, inverse: global stages L1-1..0 of GS, F folded into stage 0, canonical output.
template <class A, class TOut, int L1>
__global__ __launch_bounds__(256) void k_cols_inv(KParams<A> P,
                                                  const typename A::word *__restrict__ tc,
                                                  TOut *__restrict__ c, size_t batch, int logs) {
  using W = typename A::word;
  constexpr int M = 1 << L1;
  const size_t ncol = (size_t)1 << logs;
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= batch * ncol) return;
  const size_t p = gid >> logs, col = gid & (ncol - 1);
  const size_t base = (p << (logs + L1)) + col;
  const size_t base_r = NTTMUL_HOOK_COLS_LD(base, p, logs + L1, col, 1);
  W x[M];
#pragma clang loop unroll(full)
  for (int m = 0; m < M; m++) x[m] = ld_stream<NTTMUL_NT_COLS>(tc + base_r + ((size_t)m << logs));
#pragma clang loop unroll(full)
  for (int st = L1 - 1; st >= 0; st--) {
    const int dist = M >> (st + 1);
#pragma clang loop unroll(full)
    for (int m = 0; m < M; m++) {
      if (m & dist) continue;
      if (st == 0) {
        P.ar.gs_scaled(x[m], x[m + dist], P.f, P.fs, P.wf, P.wfs);
      } else {
        const TwPair<W> t = P.iw[(1 << st) + (m >> (L1 - st))];
        P.ar.gs(x[m], x[m + dist], t.w, t.ws);
      }
    }
  }
#pragma clang loop unroll(full)
  for (int m = 0; m < M; m++)
    st_stream<NTTMUL_NT_COLS>(c + base + ((size_t)m << logs),
                              (TOut)(A::kInvCanonical ? x[m] : P.ar.canon_inv(x[m])));
}

// Column pass of the square split n = 2^8 x 2^8 (n = 65536, NTTMUL_C5_SQ): each column of 256
// coefficients (stride 256 words) is a 256-point transform of global stages 0..7, run like one
// k_rows row of Groups<8> (16 coefficients per thread, two register groups of four stages, one LDS
// exchange) on the column's elements m = 0..255 (address m * 256 + column).  A 256-thread
// workgroup takes 16 adjacent columns: thread t = 16 jj + cl runs register-group position jj of
// column cl, so every load and store instruction moves 4 rows x 16 columns (128-B runs for u64),
// and the 16 transforms share the LDS element by element (word 16 padx(e) + cl: conflict-free for
// ds_write_b64's 16-lane and ds_read_b64's 32-lane groups).  Against the 16 x 4096
// split the VALU-bound row pass sheds half of its butterflies to these passes, which are HBM-bound
// and had VALU issue to spare.
//   DIR 0: global stages 0..7 of the forward CT on a and b (twiddles P.fw[1 .. 255], uniform over
//          the columns); X of stage 0 canonical by contract; output lazy, in place of the column
//   DIR 1: global stages 7..0 of the inverse GS with F folded into stage 0; canonical output
// NPOLY: polynomials per column group (2: a and b of a product; 1: a standalone forward transform)
template <class A, class TIn, class TOut, int DIR, int NPOLY = DIR == 0 ? 2 : 1>
__global__ __launch_bounds__(256) void k_cols8(KParams<A> P, const TIn *__restrict__ a,
                                               const TIn *__restrict__ b, TOut *__restrict__ ta,
                                               TOut *__restrict__ tb, size_t groups) {
  using W = typename A::word;
  using Gr = Groups<8>;
  constexpr int CW = 16, G = Gr::G;
  static_assert(DIR == 0 || NPOLY == 1, "the inverse column pass runs on c alone");
  constexpr int GIN = DIR == 0 ? 0 : G - 1, GOUT = DIR == 0 ? G - 1 : 0;
  static_assert(G == 2 && Gr::NP * CW >= (Gr::padx<0>(255) + 1) * CW, "Groups<8> layout");
  __shared__ W lds[Gr::NP * CW];
  const size_t g = blockIdx.x;
  if (g >= groups) return;  // (grid = groups exactly; block-uniform)
  const int cl = threadIdx.x % CW, jj = threadIdx.x / CW;
  const size_t p = g >> 4;
  const size_t base = (p << 16) + ((g & 15) << 4) + cl;  // element m of the column at base + 256 m
  // the intermediate side (DIR 0 stores, DIR 1 loads): with c8_tile the workgroup's 16 columns
  // are one contiguous 4096-word tile, element m of column cl at 16 m + cl
  constexpr bool kTile = c8_tile(8, 8);
  const size_t ibase = kTile ? (p << 16) + ((g & 15) << 12) + cl : base;
  constexpr int kIS = kTile ? 4 : 8;  // log2 word stride of m on the intermediate side
  const size_t base_r = NTTMUL_HOOK_COLS_LD(DIR == 0 ? base : ibase, p, 16, ((g & 15) << 4) + cl, DIR);
  W x[16], y[16];
  // NTTMUL_C5_BUF: one descriptor per polynomial (p is block-uniform), lane offsets relative to
  // it (< 512 KiB), each register's constant offset as the scalar offset
  constexpr bool kBuf = NTTMUL_C5_BUF && !NTTMUL_COLS_HOOKED && sizeof(TIn) == 8 &&
                        sizeof(TOut) == 8 && NTTMUL_NT_COLS;
  constexpr int kAuxB = 2;  // nt
  const size_t pbase = p << 16;
  if constexpr (kBuf) {
    const auto ra = span_rsrc(a + pbase, 65536), rb = span_rsrc(b + pbase, 65536);
    const int lane = (int)((DIR == 0 ? base : ibase) - pbase) +
                     (Gr::base(GIN, jj) << (DIR == 0 ? 8 : kIS));
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int so = (Gr::off(GIN, k) << (DIR == 0 ? 8 : kIS)) * 8;
      x[k] = (W)buf_ld64<kAuxB>(ra, lane * 8, so);
      y[k] = NPOLY == 2 ? (W)buf_ld64<kAuxB>(rb, lane * 8, so) : W(0);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const size_t o = (size_t)(Gr::base(GIN, jj) + Gr::off(GIN, k)) << (DIR == 0 ? 8 : kIS);
      x[k] = (W)ld_stream<NTTMUL_NT_COLS>(a + base_r + o);
      y[k] = NPOLY == 2 ? (W)ld_stream<NTTMUL_NT_COLS>(b + base_r + o) : W(0);
    }
  }
  if constexpr (DIR == 0) {
    TwPair<W> zw[16];
    fwd_all<A, 8, 0, NPOLY, 0, 0, CW>(P.ar, x, y, lds + cl, lds + cl, P.fw, jj, 0, 0, zw);
    if constexpr (kBuf) {
      const auto rta = span_rsrc(ta + pbase, 65536), rtb = span_rsrc(tb + pbase, 65536);
      const int lane = (int)(ibase - pbase) + (Gr::base(GOUT, jj) << kIS);
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const int so = (Gr::off(GOUT, k) << kIS) * 8;
        buf_st64<kAuxB>(rta, lane * 8, (uint64_t)x[k], so);
        if (NPOLY == 2) buf_st64<kAuxB>(rtb, lane * 8, (uint64_t)y[k], so);
      }
      return;
    }
    const size_t base_w = NTTMUL_HOOK_COLS_ST(ibase, p, 16, ((g & 15) << 4) + cl);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const size_t o = (size_t)(Gr::base(GOUT, jj) + Gr::off(GOUT, k)) << kIS;
      st_stream<NTTMUL_NT_COLS>(ta + base_w + o, (TOut)x[k]);
      if (NPOLY == 2) st_stream<NTTMUL_NT_COLS>(tb + base_w + o, (TOut)y[k]);
    }
  } else {
    inv_all<A, 8, G - 1, true, 0, 0, 1, CW>(P, x, y, lds + cl, lds + cl, P.iw, jj, 0, 0);
    if constexpr (kBuf) {
      const auto rc = span_rsrc(ta + pbase, 65536);
      const int lane = (int)(base - pbase) + (Gr::base(GOUT, jj) << 8);
#pragma unroll
      for (int k = 0; k < 16; k++)
        buf_st64<kAuxB>(rc, lane * 8, (uint64_t)(A::kInvCanonical ? x[k] : P.ar.canon_inv(x[k])),
                        (Gr::off(GOUT, k) << 8) * 8);
      return;
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const size_t o = (size_t)(Gr::base(GOUT, jj) + Gr::off(GOUT, k)) << 8;
      st_stream<NTTMUL_NT_COLS>(ta + base + o,
                                (TOut)(A::kInvCanonical ? x[k] : P.ar.canon_inv(x[k])));
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Synthetic inputs and input validation
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <class T>
__global__ void k_fill(T *a, T *b, uint32_t logn, uint64_t q, uint64_t seed, uint64_t p0,
                       size_t total) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const uint64_t n = 1ull << logn;
  const uint64_t p = i >> logn, k = i & (n - 1);
  const uint64_t base = seed + 2ull * n * (p0 + p);
  a[i] = (T)(splitmix64(base + k) % q);
  b[i] = (T)(splitmix64(base + n + k) % q);
}

// Bit-reversal permutation of each polynomial (NTT/ntt.C:27-44 bitrev_shuffle): turns the
// std2rev transforms into the reference's rev2std variants and back (ntt256.h:20-69).
template <class T>
__global__ void k_bitrev(const T *__restrict__ in, T *__restrict__ out, uint32_t logn,
                         size_t total) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const size_t e = i & ((1u << logn) - 1), p = i - e;
  out[p + (__brev((uint32_t)e) >> (32 - logn))] = in[i];
}
template <class T>
__global__ void k_bitrev_inplace(T *a, uint32_t logn, size_t total) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const size_t e = i & ((1u << logn) - 1), p = i - e;
  const size_t r = __brev((uint32_t)e) >> (32 - logn);
  if (e < r) {
    const T t = a[p + e];
    a[p + e] = a[p + r];
    a[p + r] = t;
  }
}

template <class T>
__global__ void k_check_range(const T *a, const T *b, uint64_t q, size_t total, int *bad) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  if ((uint64_t)a[i] >= q || (uint64_t)b[i] >= q) atomicOr(bad, 1);
}

// ---------------------------------------------------------------------------------------------
// Launch helpers shared by the library's dispatch (kernels.hip) and tools/kbench
// ---------------------------------------------------------------------------------------------
template <class A>
static KParams<A> make_params(const LaunchTables &T) {
  using W = typename A::word;
  KParams<A> P;
  P.ar.q = (W)T.q;
  P.ar.qinv_neg = (W)T.qinv_neg;
  if constexpr (std::is_same<A, Arith64>::value) P.ar.q2 = 2 * T.q;
  if constexpr (IsPlantard<A>::value) {
    P.ar.c32 = (uint32_t)((1ull << 32) % T.q);
    P.ar.as = (uint32_t)((3 * T.q + 1) / 2);
  }
  P.fw = (const TwPair<W> *)T.fw;
  P.iw = (const TwPair<W> *)T.iw;
  P.f = (W)T.f; P.fs = (W)T.fs; P.wf = (W)T.wf; P.wfs = (W)T.wfs;
  return P;
}

// KParams for the product kernels: with incomplete transforms the inverse skips D stages and
// leaves (n / 2^D) c, so the folded scale is F 2^D
template <class A>
static KParams<A> product_params(const LaunchTables &T) {
  using W = typename A::word;
  KParams<A> P = make_params<A>(T);
  static_assert(A::kBaseD == 0 || A::kBaseD == 2 || A::kBaseD == 3,
                "planner provides F 2^D for D = 2, 3");
  if (NTTMUL_BASE_D && A::kBaseD == 2) {
    P.f = (W)T.f4; P.fs = (W)T.f4s; P.wf = (W)T.wf4; P.wfs = (W)T.wf4s;
  } else if (NTTMUL_BASE_D && A::kBaseD == 3) {
    P.f = (W)T.f8; P.fs = (W)T.f8s; P.wf = (W)T.wf8; P.wfs = (W)T.wf8s;
  }
  return P;
}

// Issue priority of the fused product (k_rows, L1 = 0).  The wave scheduler issues the oldest
// ready wave first, so of the waves a SIMD holds the first finishes long before the last, which
// then runs its tail alone with no other wave to hide its latencies: at C2 (n = 1024 x 4096, one
// generation of 4 waves per SIMD) the four waves of a SIMD computed in 7.1 / 9.3 / 11.8 / 14.5 us
// (tools/kbench per-SIMD trace, profiles/r3/c2/wave_trace_slots.txt).  With P.prio each wave
// drops its priority as it completes phases (3 for the forward transforms, 1 for the base
// multiplication, 0 for the inverse; k_rows<..., PRIO = true>), so the waves that are behind
// issue first and all finish together: C2 17.6 vs 18.6 us; n = 512 x 8192, 256 x 16384, 2048 x 2048, 4096 x 1024 +4..9 %
// (profiles/r3/c2/prio_ab2.txt).  It only pays when the launch is one thin generation: at 8
// waves per SIMD (n = 1024 x 8192, 4096 x 2048) or many generations (C3, 1024 x 262144) the
// oldest-first order is 1-7 % faster (a finished wave frees its slot early, and the loads of the
// next block overlap the others' arithmetic).  So: on when the launch has at most 4 waves per
// SIMD of the device and the previous product launch of the context went to the same stream
// (T.prio_ok, nttmul.cpp run_device: launches alternating over two streams overlap, and then the
// oldest-first order wins, 292 vs 262 M/s at C2); nttmul_params.issue_prio -1 / 1 forces it off /
// on for a context.
static thread_local int tl_prio_cus = 0;   // launch_polymul: T.cus, or 0 when T.prio_ok is 0
static thread_local int tl_prio_mode = 0;  // launch_polymul: T.prio (nttmul_params.issue_prio)
static bool rows_prio(size_t waves) {
  if (tl_prio_mode) return tl_prio_mode > 0;
  return waves <= (size_t)tl_prio_cus * 4 * 4;  // 4 SIMDs per CU, 4 waves per SIMD
}

template <class A, class TIn, class TOut, int LOGS, int L1>
static hipError_t launch_rows(const KParams<A> &P, const void *a, const void *b, void *c,
                              size_t units, hipStream_t s) {
  constexpr int NT = rows_threads(LOGS), PB = NT / ((1 << LOGS) / 16);
  const size_t blocks = (units + PB - 1) / PB;
  // (the prioritised variant exists for the u32 Plantard products only: q < 2^31, C2 / C3 family)
  constexpr bool kPrioOk = L1 == 0 && IsPlantard<A>::value && sizeof(TIn) == 4 && sizeof(TOut) == 4;
  const bool prio = kPrioOk && blocks && rows_prio(blocks * (NT / 64));
  if (tl_describe) {
    describe_add(std::string("k_rows<") + AName<A>::v + "," + word_name<TIn>() + "," +
                 word_name<TOut>() + "," + std::to_string(LOGS) + "," + std::to_string(L1) +
                 (prio ? ",prio>" : ">"));
    return hipSuccess;
  }
  if (blocks == 0) return hipSuccess;
  if constexpr (kPrioOk) {
    if (prio) {
      hipLaunchKernelGGL((k_rows<A, TIn, TOut, LOGS, L1, true>), dim3((unsigned)blocks), dim3(NT), 0,
                         s, P, (const TIn *)a, (const TIn *)b, (TOut *)c, units);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((k_rows<A, TIn, TOut, LOGS, L1>), dim3((unsigned)blocks), dim3(NT), 0, s, P,
                     (const TIn *)a, (const TIn *)b, (TOut *)c, units);
  return hipGetLastError();
}


}  // namespace nttmul
