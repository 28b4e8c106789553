// modarith.hpp — device-side modular arithmetic for the NTT kernels (gfx950).
//
// Replaces the reference's Q=12289-specialised arithmetic (NTT/ntt.C:69-107 add_mod/sub_mod/
// divq/modq; NTT-RED/ntt_red.c:34-46 K-RED) with word-size-generic lazy Shoup butterflies:
//
//   Arith32 : q < 2^31, values kept in [0, 2q) inside 32-bit registers.  A twiddle product is
//             one v_mul_lo_u32 + two v_mad_u64_u32 with the twiddle in Montgomery form (or,
//             NTTMUL_A32_MONT=0, Shoup: v_mul_hi_u32 + two v_mul_lo_u32 + v_sub); a conditional
//             subtraction is v_sub_co_u32 + v_cndmask_b32 (no compare/branch).
//   Arith32W: 2^31 <= q < 2^32, canonical values, Montgomery twiddles with a 65-bit sum.
//   Arith64 : q < 2^62, values lazy in 64-bit registers, 64x64 Shoup in 32-bit limbs.
//
// Pointwise products use Montgomery (R = 2^32 or 2^64); the R^-1 it introduces and the n^-1 of
// the inverse transform are folded into one constant F = n^-1 R (mod q) applied in the last
// inverse stage, so the product needs no separate scaling pass (the reference's final
// mul_array16 by scaled_inv_psi_powers, NTT/ntt256.C:12, disappears into the twiddles).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arith_select.hpp"

// conditional-subtract lowering: 0 = e32 sub_co/cndmask asm, 1 = v_min_u32,
// 2 = __builtin_sub_overflow + select (default: measured fastest in k_rows, tools/kbench)
#ifndef NTTMUL_CSUB
#define NTTMUL_CSUB 2
#endif
// typed P/N butterflies for Arith32 (q < 2^31): 1 = on (needs the planner's centred tables)
#ifndef NTTMUL_TYPED
#define NTTMUL_TYPED 1
#endif
// Arith32 twiddle products: 0 = Shoup (w, floor(w 2^32 / q)), 1 = Montgomery form (planner.cpp
// emits the matching table pairs; the macro must agree between host and device objects)
#ifndef NTTMUL_A32_MONT
#define NTTMUL_A32_MONT 1
#endif
// Arith32 twiddle products as Seiler's signed Montgomery (v_mul_lo + 2 v_mul_hi + v_sub, no
// carry-out SGPR writes); the planner then stores -w2 (A/B variant, untyped butterflies only)
#ifndef NTTMUL_A32_SEILER
#define NTTMUL_A32_SEILER 0
#endif
#if NTTMUL_A32_SEILER && NTTMUL_TYPED
#error "NTTMUL_A32_SEILER needs NTTMUL_TYPED=0"
#endif

namespace nttmul {

// H (Harvey lazy bounds, q < 2^30): forward values in [0, 4q), inverse values in [0, 2q), one
// conditional subtraction per butterfly instead of two.  Without H (q < 2^31) there is no
// headroom above 2q in a 32-bit word and every butterfly reduces both of its operands.
template <bool H>
struct Arith32T {
  using word = uint32_t;
  static constexpr int kBits = 32;
  // typed butterflies (kernels.hip fwd_group / inv_group): see ct_t below
  static constexpr bool kTyped = !H && NTTMUL_TYPED && NTTMUL_A32_MONT;
  static constexpr bool kInvCanonical = false;  // inverse outputs lazy: canonicalised at the store
  uint32_t q;
  uint32_t qinv_neg;  // -q^-1 mod 2^32

  // x in [0, 2m) -> [0, m).  Written as subtract-with-borrow + select so hipcc emits
  // v_sub_co_u32 + v_cndmask_b32 (both full-rate on gfx950, ~2.4 cycles per wave64 instruction)
  // instead of v_sub + v_min_u32 (v_min_u32 issues at ~4.2 cycles; tools/microbench/valu_issue).
  __device__ __forceinline__ static uint32_t csub(uint32_t x, uint32_t m) {
#if NTTMUL_CSUB == 1
    return min(x, x - m);
#elif NTTMUL_CSUB == 2
    uint32_t d;
    return __builtin_sub_overflow(x, m, &d) ? x : d;
#elif NTTMUL_CSUB == 3
    // sign-mask form (m < 2^31, so x - m is a valid int32): v_sub + v_ashr + v_and + v_add
    // (the shift is opaque asm so the compiler cannot fold the mask back into cmp + cndmask)
    const uint32_t d = x - m;
    uint32_t s;
    asm("v_ashrrev_i32_e32 %0, 31, %1" : "=v"(s) : "v"(d));
    return d + (s & m);
#else
    // VOP2 (e32) forms through VCC: the VOP3 forms with an SGPR-pair carry/mask that hipcc
    // otherwise picks issue at ~4.3 cycles each on gfx950, the e32 pair at ~2.4.  The s_nop
    // covers the VALU-writes-VCC -> VALU-reads-VCC hazard; other waves issue meanwhile.
    uint32_t r;
    asm("v_subrev_co_u32_e32 %0, vcc, %2, %1\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e32 %0, %0, %1, vcc"
        : "=&v"(r)
        : "v"(x), "s"(m)
        : "vcc");
    return r;
#endif
  }

#if NTTMUL_A32_SEILER
  // x w 2^-32 in (-q, q) for any 32-bit x: m = x w2n with w2n = w1 q^-1 mod 2^32, so x w1 and
  // m q agree in their low words and the difference of the high words is exact
  __device__ __forceinline__ uint32_t mont_sl(uint32_t x, uint32_t w1, uint32_t w2n) const {
    const uint32_t m = x * w2n;
    return __umulhi(x, w1) - __umulhi(m, q);
  }
  __device__ __forceinline__ uint32_t shoup(uint32_t x, uint32_t w1, uint32_t w2n) const {
    return mont_sl(x, w1, w2n) + q;  // [0, 2q)
  }
  // (-q, q) -> [0, q) without a carry: t + q wraps to the small value exactly when t < 0
  __device__ __forceinline__ static uint32_t fold(uint32_t t, uint32_t m) { return min(t, t + m); }
#elif NTTMUL_A32_MONT
  // x * w mod q in [0, 2q) for any 32-bit x, twiddle in Montgomery form (w1 = w 2^32 mod q,
  // w2 = w1 (-q^-1) mod 2^32): (x w1 + m q) / 2^32 with m = x w2 mod 2^32 — one v_mul_lo_u32
  // and two v_mad_u64_u32, no trailing subtraction.  x w1 + m q < 2^33 q < 2^64 for q < 2^31.
  __device__ __forceinline__ uint32_t shoup(uint32_t x, uint32_t w1, uint32_t w2) const {
    const uint32_t m = x * w2;
    const uint64_t s = (uint64_t)x * w1 + (uint64_t)m * q;
    return (uint32_t)(s >> 32);
  }
#else
  // x * w mod q in [0, 2q) for any 32-bit x (Shoup).
  __device__ __forceinline__ uint32_t shoup(uint32_t x, uint32_t w, uint32_t ws) const {
    uint32_t qh = __umulhi(x, ws);
    return x * w - qh * q;
  }
#endif
#if NTTMUL_A32_MONT
  // --- typed butterflies (q < 2^31, Montgomery twiddles) -------------------------------------
  // A register holds a P-type value in [0, 2q) (unsigned) or an N-type value in (-q, q) (int32).
  // Inside a register group every operand's type is a compile-time fact (bit 2 dist of the
  // register index says whether the previous stage wrote it as X or Y), so the CT difference
  // x - t and the GS difference x - y can stay N-type instead of paying "+ q" to stay
  // non-negative: one VALU instruction less per butterfly.  N-type operands are reduced by
  // cadd (the carry of y + q is the sign of y) and multiplied by mont_s with the centred
  // twiddle (w1 in (-q/2, q/2], planner.cpp appends that table after the unsigned one).
  // Group boundaries (LDS exchanges, the base multiplication, stores) see P-type only.
  __device__ __forceinline__ static uint32_t cadd(uint32_t x, uint32_t m) {
    uint32_t e;
    return __builtin_add_overflow(x, m, &e) ? e : x;
  }
  template <bool N>
  __device__ __forceinline__ uint32_t corr(uint32_t x) const {
    return N ? cadd(x, q) : csub(x, q);
  }
  // y w mod q for y in (-q, q) (int32) and the centred Montgomery pair (w1c, w2c = w1c (-q^-1)):
  // |y w1c + m q| < q^2 / 2 + 2^31 q, so the result lies in (-0.74 q, 0.74 q).
  __device__ __forceinline__ uint32_t mont_s(uint32_t y, uint32_t w1c, uint32_t w2c) const {
    const int32_t m = (int32_t)(y * w2c);
    const int64_t s = (int64_t)(int32_t)y * (int32_t)w1c + (int64_t)m * (int32_t)q;
    return (uint32_t)(int32_t)(s >> 32);
  }
  // CT on operands of type IN_N (X and Y share it); (w, ws) is the centred pair when IN_N.
  // Outputs: X' P-type, Y' N-type (OUT_P: P-type, x - t + q, at the end of a register group).
  template <bool IN_N, bool OUT_P, bool XC = false>
  __device__ __forceinline__ void ct_t(uint32_t &X, uint32_t &Y, uint32_t w, uint32_t ws) const {
    const uint32_t x = XC ? X : corr<IN_N>(X);
    const uint32_t t = IN_N ? cadd(mont_s(Y, w, ws), q) : csub(shoup(Y, w, ws), q);
    X = x + t;
    Y = OUT_P ? x - t + q : x - t;
  }
  // GS on operands of type IN_N; (w, ws) centred unless OUT_P.  X' P-type, Y' N-type in
  // (-0.74 q, 0.74 q) (OUT_P: P-type).
  template <bool IN_N, bool OUT_P>
  __device__ __forceinline__ void gs_t(uint32_t &X, uint32_t &Y, uint32_t w, uint32_t ws) const {
    const uint32_t x = corr<IN_N>(X), y = corr<IN_N>(Y);
    X = x + y;
    Y = OUT_P ? shoup(x - y + q, w, ws) : mont_s(x - y, w, ws);
  }
  template <bool IN_N>
  __device__ __forceinline__ void gs_scaled_t(uint32_t &X, uint32_t &Y, uint32_t f, uint32_t fs,
                                              uint32_t wf, uint32_t wfs) const {
    const uint32_t x = corr<IN_N>(X), y = corr<IN_N>(Y);
    X = shoup(x + y, f, fs);
    Y = shoup(x - y + q, wf, wfs);
  }
#endif
  // Cooley-Tukey butterfly, ntt.C:365-367 pattern: (X, Y) -> (X + Y w, X - Y w).  In/out [0, 2q);
  // XC: X is known canonical (the first stage of a transform of canonical input).
  // (H: X in [0, 4q), outputs in [0, 4q).)
  template <bool XC = false>
  __device__ __forceinline__ void ct(uint32_t &X, uint32_t &Y, uint32_t w, uint32_t ws) const {
    if (H) {
      const uint32_t x = XC ? X : csub(X, 2 * q);
      const uint32_t t = shoup(Y, w, ws);
      X = x + t;
      Y = x - t + 2 * q;
      return;
    }
    uint32_t x = XC ? X : csub(X, q);
#if NTTMUL_A32_SEILER
    uint32_t t = fold(mont_sl(Y, w, ws), q);
#else
    uint32_t t = csub(shoup(Y, w, ws), q);
#endif
    X = x + t;
    Y = x - t + q;
  }
  // Gentleman-Sande butterfly, ntt.C:445-447 pattern: (X, Y) -> (X + Y, (X - Y) w).  In/out [0, 2q).
  __device__ __forceinline__ void gs(uint32_t &X, uint32_t &Y, uint32_t w, uint32_t ws) const {
    if (H) {
      const uint32_t x = X, y = Y;
      X = csub(x + y, 2 * q);
      Y = shoup(x - y + 2 * q, w, ws);
      return;
    }
    uint32_t x = csub(X, q), y = csub(Y, q);
    X = x + y;
    Y = shoup(x - y + q, w, ws);
  }
  // Last inverse stage with the output scale F folded in: (X, Y) -> ((X + Y) F, (X - Y) w F).
  __device__ __forceinline__ void gs_scaled(uint32_t &X, uint32_t &Y, uint32_t f, uint32_t fs,
                                            uint32_t wf, uint32_t wfs) const {
    if (H) {
      const uint32_t x = X, y = Y;
      X = shoup(x + y, f, fs);
      Y = shoup(x - y + 2 * q, wf, wfs);
      return;
    }
    uint32_t x = csub(X, q), y = csub(Y, q);
    X = shoup(x + y, f, fs);
    Y = shoup(x - y + q, wf, wfs);
  }
  // Montgomery product a b 2^-32 mod q, inputs lazy (H: < 4q, else < 2q), output in [0, 2q).
  // H: both reduced below 2q, t + m q < 4 q^2 + 2^32 q < 2^64.  Otherwise only a is reduced
  // (below q): a b + m q < 2 q^2 + 2^32 q < 2^64 and (a b + m q) / 2^32 < q (2q / 2^32 + 1) < 2q.
  __device__ __forceinline__ uint32_t mont(uint32_t a, uint32_t b) const {
    const uint32_t ar = H ? csub(a, 2 * q) : csub(a, q), br = H ? csub(b, 2 * q) : b;
    uint64_t t = (uint64_t)ar * br;
    uint32_t m = (uint32_t)t * qinv_neg;
    uint64_t u = t + (uint64_t)m * q;
    return (uint32_t)(u >> 32);
  }
  // lazy -> [0, q)
  __device__ __forceinline__ uint32_t canon(uint32_t x) const {
    return H ? csub(csub(x, 2 * q), q) : csub(x, q);
  }
  // an inverse transform's output -> [0, q) (see Arith64::canon_inv; unchanged here)
  __device__ __forceinline__ uint32_t canon_inv(uint32_t x) const { return canon(x); }

  // Base multiplication of the incomplete transform (kernels.hip base_mult): a = a b 2^-32 in
  // Z_q[x]/(x^B - z), z = (NEG ? -1 : 1) w for the Montgomery-form twiddle (w1, w2).  Inputs
  // lazy (forward-transform bounds), output in [0, 2q) like mont().  Schoolbook over 64-bit
  // accumulators, one Montgomery reduction per output coefficient; the wrapped terms use
  // b'_i = z b_i (one twiddle product each).
  //   q < 2^31: a, b, b' canonical, each sum < B q^2 < 2^64 (B = 4); the Montgomery sum can
  //             reach 2^65, its carry is folded into the final conditional subtraction.
  //   H       : a < 2q, b and b' canonical, sum < 2 B q^2 < 2^63, result < 3q.
  static constexpr int kBaseD = 2;
  // ZC: (w1, w2) is the centred pair (the last forward stage multiplied N-type operands by it).
  template <int B, bool NEG, bool ZC = false>
  __device__ __forceinline__ void basemul(uint32_t (&a)[B], const uint32_t (&b)[B], uint32_t w1,
                                          uint32_t w2) const {
    static_assert(B == 4, "sums of B products must fit 64 bits");
    if (NEG && ZC) {  // -w centred: (-w1c, -w2c)
      w1 = 0u - w1;
      w2 = 0u - w2;
    } else if (NEG) {  // -w in Montgomery form: (q - w1, (q - w1)(-q^-1) = ~w2 mod 2^32)
      w1 = q - w1;
#if NTTMUL_A32_SEILER
      w2 = 1u - w2;     // (q - w1) q^-1 = 1 - w1 q^-1
#else
      w2 = ~w2;
#endif
    }
    uint32_t ar[B], br[B], bz[B];
#pragma unroll
    for (int i = 0; i < B; i++) {
      ar[i] = H ? csub(a[i], 2 * q) : csub(a[i], q);
      br[i] = H ? csub(csub(b[i], 2 * q), q) : csub(b[i], q);
    }
#pragma unroll
    for (int i = 1; i < B; i++) {
#if NTTMUL_A32_MONT
      if (ZC && !H) {
        bz[i] = cadd(mont_s(br[i], w1, w2), q);
        continue;
      }
#endif
      bz[i] = csub(shoup(b[i], w1, w2), q);
    }
#pragma unroll
    for (int k = 0; k < B; k++) {
      uint64_t s = 0;
#pragma unroll
      for (int i = 0; i < B; i++)
        s += (uint64_t)ar[i] * (i <= k ? br[k - i] : bz[B + k - i]);
      const uint32_t m = (uint32_t)s * qinv_neg;
      if (H) {
        a[k] = csub((uint32_t)((s + (uint64_t)m * q) >> 32), 2 * q);
      } else {
        uint64_t t;
        const bool c = __builtin_add_overflow(s, (uint64_t)m * q, &t);  // value c 2^64 + t
        const uint32_t hi = (uint32_t)(t >> 32);                      // result < 2.875 q
        uint32_t d;
        const bool br2 = __builtin_sub_overflow(hi, 2 * q, &d);
        a[k] = (c || !br2) ? d : hi;
      }
    }
  }
};
using Arith32 = Arith32T<false>;   // q < 2^31
using Arith32H = Arith32T<true>;   // q < 2^30

// q < 2^31 with Plantard twiddle products (T. Plantard, "Efficient word size modular arithmetic",
// IEEE TETC 2021).  The twiddle w is stored as BR = B q^-1 mod 2^64 with B = -w 2^64 mod q, split
// (b0, b1) = (low, high) word.  For any 32-bit x:
//   T = x BR mod 2^64,  t = floor((floor(T / 2^32) + 1) q / 2^32)
// k = (T q - x B) / 2^64 is an integer in [0, q) congruent to -x B 2^-64 = x w, and
// t = floor(k + e) with e = (x B + (2^32 - T mod 2^32) q) / 2^64 in (0, 1) whenever
// x B < 2^32 (2^32 - q), which holds for every 32-bit x and B < q because 2q < 2^32.  So t is
// the canonical residue of x w, for one v_mul_hi_u32 + v_mul_lo_u32 + v_add_u32 +
// v_mad_u64_u32 — the same three multiplies as a Montgomery product, whose output spans [0, 2q)
// and needs a conditional subtraction (two carry/select instructions) before it can be added.
// Butterflies therefore correct one operand instead of two:
//   CT  (forward, x lazy in [0, 2q), Y any word): x = csub(X); t = x w; (x + t, x - t + q)
//   GS  (inverse, x, y canonical): (csub(x + y), (x - y + q) w), both outputs canonical
// Every inverse value is canonical, so the transform's output needs no final canonicalisation.
// NTTMUL_P_TYPED (Arith32P CT differences kept signed): arith_select.hpp
#ifndef NTTMUL_P_HI  // Arith32P: last Plantard step as v_mul_hi_u32(th + 1, q) (A/B variant)
#define NTTMUL_P_HI 0
#endif
#ifndef NTTMUL_P_FOLD  // Arith32P base multiplication: fold the sum's high word by 2^32 mod q
#define NTTMUL_P_FOLD 1
#endif
#ifndef NTTMUL_P3_PIN  // Arith32P3 base multiplication: pin the halfway fold (empty asm)
#define NTTMUL_P3_PIN 1
#endif
struct Arith32P {
  using word = uint32_t;
  static constexpr int kBits = 32;
  static constexpr bool kTyped = false;
  static constexpr bool kTypedP = NTTMUL_P_TYPED;  // kernels.hip fwd_group: ct<XC, XN, YN>
  static constexpr bool kInvCanonical = true;  // GS outputs are canonical
  uint32_t q;
  uint32_t qinv_neg;  // -q^-1 mod 2^32 (Montgomery reduction of the base-multiplication sums)
  uint32_t c32;       // 2^32 mod q
  uint32_t as;        // ceil(1.5 q): the signed-input Plantard addend (pmul_s)

  __device__ __forceinline__ static uint32_t csub(uint32_t x, uint32_t m) {
    uint32_t d;
    return __builtin_sub_overflow(x, m, &d) ? x : d;
  }
  // int32 x in (-q, q) -> [0, q): the carry of x + q is set exactly when x < 0
  __device__ __forceinline__ uint32_t cadd(uint32_t x) const {
    uint32_t e;
    return __builtin_add_overflow(x, q, &e) ? e : x;
  }
  // x w mod q in [0, q) for any 32-bit x; (b0, b1) = the planner's Plantard pair of w
  __device__ __forceinline__ uint32_t pmul(uint32_t x, uint32_t b0, uint32_t b1) const {
    const uint32_t th = __umulhi(x, b0) + x * b1;
#if NTTMUL_P_HI
    // th + 1 never wraps: th = 2^32 - 1 would give t = q, and t < q
    return __umulhi(th + 1, q);
#else
    return (uint32_t)(((uint64_t)th * q + q) >> 32);
#endif
  }
  // x w mod q in [0, q) for int32 x in (-q, q) (also any int32 but -q, -2q...), with the
  // signed pair (b0, b1 + (b0 >> 31)) of the planner: T = x BR mod 2^64 through v_mul_hi_i32, and
  // t = floor((T_hi q + A) / 2^32) is exact for A in [q + 2^31 q / 2^32, 2^32 - 2^31 q / 2^32),
  // non-empty for q < 2^31 (the error term spans 2^32 q < 2^32 (2^32 - q)); A = ceil(1.5 q)
  // ASM: the signed high product as opaque inline asm -- for a stage compiled twice behind a
  // wave-uniform branch (kernels.hip fwd_stage, TIN), where the optimizer would otherwise merge
  // the two copies' high products into one 64-bit multiply with selects
  template <bool ASM = false>
  __device__ __forceinline__ uint32_t pmul_s(uint32_t x, uint32_t b0, uint32_t b1s) const {
    uint32_t hi;
    if constexpr (ASM)
      asm volatile("v_mul_hi_i32 %0, %1, %2" : "=v"(hi) : "v"(x), "v"(b0));
    else
      hi = (uint32_t)__mulhi((int)x, (int)b0);
    const uint32_t th = hi + x * b1s;
    return (uint32_t)(((uint64_t)th * q + as) >> 32);
  }
  __device__ __forceinline__ uint32_t shoup(uint32_t x, uint32_t b0, uint32_t b1) const {
    return pmul(x, b0, b1);
  }
  // inverse-table product of a GS difference x - y (x, y canonical)
  __device__ __forceinline__ uint32_t pmul_diff(uint32_t x, uint32_t y, uint32_t b0,
                                                uint32_t b1) const {
#if NTTMUL_P_SIGNED_INV
    return pmul_s(x - y, b0, b1);
#else
    return pmul(x - y + q, b0, b1);
#endif
  }
  // CT (ntt.C:365-367 pattern): X in [0, 2q) (XC: canonical; XN: signed in (-q, q)), Y any ->
  // X' in [0, 2q), Y' in (0, 2q) (YN: x - t signed in (-q, q), for a register whose next use is
  // as the X of a butterfly, where the carry of x + q corrects it as cheaply as csub would)
  template <bool XC = false, bool XN = false, bool YN = false, bool ASM = false>
  __device__ __forceinline__ void ct(uint32_t &X, uint32_t &Y, uint32_t b0, uint32_t b1) const {
    uint32_t x;
    if (XC) {
      x = X;
    } else if (XN) {
      uint32_t e;
      x = __builtin_add_overflow(X, q, &e) ? e : X;
    } else {
      x = csub(X, q);
    }
    // NTTMUL_P_TYPED 2: an N-type X comes with an N-type Y and a signed-form twiddle pair
    const uint32_t t = XN && NTTMUL_P_TYPED >= 2 ? pmul_s<ASM>(Y, b0, b1) : pmul(Y, b0, b1);
    X = x + t;
    Y = YN ? x - t : x - t + q;
  }
  // GS (ntt.C:445-447 pattern): X, Y canonical -> outputs canonical
  __device__ __forceinline__ void gs(uint32_t &X, uint32_t &Y, uint32_t b0, uint32_t b1) const {
    const uint32_t x = X, y = Y;
    X = csub(x + y, q);
    Y = pmul_diff(x, y, b0, b1);
  }
  // last inverse stage with the output scale F folded in: ((X + Y) F, (X - Y) w F), canonical
  __device__ __forceinline__ void gs_scaled(uint32_t &X, uint32_t &Y, uint32_t f0, uint32_t f1,
                                            uint32_t wf0, uint32_t wf1) const {
    const uint32_t x = X, y = Y;
    X = pmul(x + y, f0, f1);
    Y = pmul_diff(x, y, wf0, wf1);
  }
  // Montgomery a b 2^-32 mod q, a and b in [0, 2q) -> [0, q): a reduced below q, so
  // a b + m q < 2 q^2 + 2^32 q < 2^64 and the quotient is below 2q
  __device__ __forceinline__ uint32_t mont(uint32_t a, uint32_t b) const {
    const uint64_t t = (uint64_t)csub(a, q) * b;
    const uint32_t m = (uint32_t)t * qinv_neg;
    return csub((uint32_t)((t + (uint64_t)m * q) >> 32), q);
  }
  // [0, 2q) -> [0, q)
  __device__ __forceinline__ uint32_t canon(uint32_t x) const { return csub(x, q); }
  __device__ __forceinline__ uint32_t canon_inv(uint32_t x) const { return csub(x, q); }

  // Base multiplication (see Arith32T::basemul): a = a b 2^-32 in Z_q[x]/(x^4 - z), z = +-w.
  // a, b in [0, 2q) from the forward transform; z b_i by Plantard (canonical straight from any
  // b_i; -w: q - w b_i, in (0, q]); four products per output, each sum below 4 q^2 < 2^64; the
  // Montgomery quotient (carry c, word hi) is below 2.875 q and is reduced to [0, q) for the
  // inverse butterflies.
  static constexpr int kBaseD = 2;
  template <int B, bool NEG, bool ZC = false>
  __device__ __forceinline__ void basemul(uint32_t (&a)[B], const uint32_t (&b)[B], uint32_t w0,
                                          uint32_t w1) const {
    static_assert(B == 4, "sums of B products must fit 64 bits");
    // a -w block (x^4 + w) holds the last forward stage's differences: with NTTMUL_P_TYPED 2 they
    // arrive signed in (-q, q) and are corrected by the carry of x + q
    constexpr bool kN = NEG && NTTMUL_P_TYPED >= 2;
    uint32_t ar[B], br[B], bz[B];
#pragma unroll
    for (int i = 0; i < B; i++) {
      ar[i] = kN ? cadd(a[i]) : csub(a[i], q);
      br[i] = kN ? cadd(b[i]) : csub(b[i], q);
    }
#pragma unroll
    for (int i = 1; i < B; i++) {
      // ZC: the z pair is in signed form (NTTMUL_P_TYPED 2): multiply the canonical b_i
      const uint32_t t = ZC ? pmul_s(br[i], w0, w1) : pmul(kN ? br[i] : b[i], w0, w1);
      bz[i] = NEG ? q - t : t;
    }
#pragma unroll
    for (int k = 0; k < B; k++) {
      uint64_t s = 0;
#pragma unroll
      for (int i = 0; i < B; i++)
        s += (uint64_t)ar[i] * (i <= k ? br[k - i] : bz[B + k - i]);
#if NTTMUL_P_FOLD
      // s = h 2^32 + l == h c32 + l (mod q): s2 <= 4 (q-1)^3 / 2^32 + 2^32 - 1, so s2 + m q < 2^64
      // and the Montgomery quotient is below (q - 1) + 1 + q = 2q: one csub to canonical
      const uint64_t s2 = (uint64_t)(uint32_t)(s >> 32) * c32 + (uint32_t)s;
      const uint32_t m = (uint32_t)s2 * qinv_neg;
      a[k] = csub((uint32_t)((s2 + (uint64_t)m * q) >> 32), q);
#else
      const uint32_t m = (uint32_t)s * qinv_neg;
      uint64_t t;
      const bool c = __builtin_add_overflow(s, (uint64_t)m * q, &t);  // value c 2^64 + t
      const uint32_t hi = (uint32_t)(t >> 32);
      uint32_t d;
      const bool br2 = __builtin_sub_overflow(hi, 2 * q, &d);
      a[k] = csub((c || !br2) ? d : hi, q);
#endif
    }
  }
  // basemul<4, NEG, true> with NEG known per lane (kernels.hip server_wide256: one block per
  // lane): a and b of a -w block arrive as signed differences, of a +w block as lazy sums; z is
  // in signed form, which the signed-input product multiplies exactly for canonical inputs.
  __device__ __forceinline__ void basemul4_lane(uint32_t (&a)[4], const uint32_t (&b)[4],
                                                uint32_t z0, uint32_t z1s, bool neg) const {
    uint32_t ar[4], br[4], bz[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      ar[i] = neg ? cadd(a[i]) : csub(a[i], q);
      br[i] = neg ? cadd(b[i]) : csub(b[i], q);
    }
#pragma unroll
    for (int i = 1; i < 4; i++) {
      const uint32_t t = pmul_s(br[i], z0, z1s);
      bz[i] = neg ? q - t : t;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint64_t s = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) s += (uint64_t)ar[i] * (i <= k ? br[k - i] : bz[4 + k - i]);
      // (the fold and reduction of basemul, NTTMUL_P_FOLD)
      const uint64_t s2 = (uint64_t)(uint32_t)(s >> 32) * c32 + (uint32_t)s;
      const uint32_t m = (uint32_t)s2 * qinv_neg;
      a[k] = csub((uint32_t)((s2 + (uint64_t)m * q) >> 32), q);
    }
  }
};

// Arith32P with base blocks of 8 coefficients (D = 3): one butterfly stage fewer in each of the
// three transforms for a base multiplication of 8 x 8 products per block.  Each output's eight
// products of canonical values are summed in two halves: the first four (< 4 q^2) are folded by
// 2^32 mod q before the other four are added, which keeps the sum below 2^64 for every
// 2^30 < q < 2^31 (arith_select.hpp p3_fold_ok, tests/test_plantard.py); the launcher takes this
// class at n = 4096 only (the last register group must hold more than 3 stages).
struct Arith32P3 : Arith32P {
  static constexpr int kBaseD = 3;
  template <int B, bool NEG, bool ZC = false>
  __device__ __forceinline__ void basemul(uint32_t (&a)[B], const uint32_t (&b)[B], uint32_t w0,
                                          uint32_t w1) const {
    static_assert(B == 8, "D = 3 blocks");
    constexpr bool kN = NEG && NTTMUL_P_TYPED >= 2;
    uint32_t ar[B], br[B], bz[B];
#pragma unroll
    for (int i = 0; i < B; i++) {
      ar[i] = kN ? cadd(a[i]) : csub(a[i], q);
      br[i] = kN ? cadd(b[i]) : csub(b[i], q);
    }
#pragma unroll
    for (int i = 1; i < B; i++) {
      const uint32_t t = ZC ? pmul_s(br[i], w0, w1) : pmul(kN ? br[i] : b[i], w0, w1);
      bz[i] = NEG ? q - t : t;
    }
    outputs<B, 0>(a, ar, br, bz);
  }
  // output K of the 8 x 8 block (compile-time recursion over K, see kernels_dev.hpp base_mult)
  template <int B, int K>
  __device__ __forceinline__ void outputs(uint32_t (&a)[B], const uint32_t (&ar)[B],
                                          const uint32_t (&br)[B], const uint32_t (&bz)[B]) const {
    if constexpr (K < B) {
      uint64_t s = 0;
#pragma unroll
      for (int i = 0; i < B / 2; i++)
        s += (uint64_t)ar[i] * (i <= K ? br[K - i] : bz[B + K - i]);
      s = (uint64_t)(uint32_t)(s >> 32) * c32 + (uint32_t)s;
#if NTTMUL_P3_PIN
      // the folded first half is the addend of the second half's multiply-add chain; without
      // the pin LLVM re-associates the second half into a fresh chain and adds the fold after
      // it (a v_mov + v_lshl_add_u64 more per output)
      asm("" : "+v"(s));
#endif
#pragma unroll
      for (int i = B / 2; i < B; i++)
        s += (uint64_t)ar[i] * (i <= K ? br[K - i] : bz[B + K - i]);
      const uint64_t s2 = (uint64_t)(uint32_t)(s >> 32) * c32 + (uint32_t)s;
      const uint32_t m = (uint32_t)s2 * qinv_neg;
      a[K] = csub((uint32_t)((s2 + (uint64_t)m * q) >> 32), q);
      outputs<B, K + 1>(a, ar, br, bz);
    }
  }
};

// 2^31 <= q < 2^32 in 32-bit words: no room above q, so values stay canonical in [0, q) and every
// sum / difference / product is reduced completely; the 65th bit of a Montgomery sum is the
// carry of a 64-bit add.  About 14 VALU instructions per butterfly, against ~30 for taking this q
// through Arith64.
struct Arith32W {
  using word = uint32_t;
  static constexpr int kBits = 32;
  static constexpr bool kTyped = false;
  static constexpr bool kInvCanonical = false;
  uint32_t q;
  uint32_t qinv_neg;  // -q^-1 mod 2^32

  __device__ __forceinline__ uint32_t addmod(uint32_t a, uint32_t b) const {
    uint32_t s, d;
    const bool c = __builtin_add_overflow(a, b, &s);
    const bool br = __builtin_sub_overflow(s, q, &d);
    return (c || !br) ? d : s;
  }
  __device__ __forceinline__ uint32_t submod(uint32_t a, uint32_t b) const {
    uint32_t d;
    return __builtin_sub_overflow(a, b, &d) ? d + q : d;
  }
  // (p + m q) / 2^32 reduced to [0, q), for p < q^2 and m = p (-q^-1) mod 2^32 given implicitly
  __device__ __forceinline__ uint32_t redc(uint64_t p, uint32_t m) const {
    uint64_t s;
    const bool c = __builtin_add_overflow(p, (uint64_t)m * q, &s);  // < 2^65: carry = bit 64
    const uint32_t hi = (uint32_t)(s >> 32);                      // value c 2^32 + hi < 2q
    uint32_t d;
    const bool br = __builtin_sub_overflow(hi, q, &d);
    return (c || !br) ? d : hi;
  }
  // x w mod q in [0, q) for x in [0, q), twiddle in Montgomery form (w1, w2 = w1 (-q^-1))
  __device__ __forceinline__ uint32_t shoup(uint32_t x, uint32_t w1, uint32_t w2) const {
    return redc((uint64_t)x * w1, x * w2);
  }
  template <bool XC = false>
  __device__ __forceinline__ void ct(uint32_t &X, uint32_t &Y, uint32_t w, uint32_t ws) const {
    const uint32_t t = shoup(Y, w, ws);
    const uint32_t x = X;
    X = addmod(x, t);
    Y = submod(x, t);
  }
  __device__ __forceinline__ void gs(uint32_t &X, uint32_t &Y, uint32_t w, uint32_t ws) const {
    const uint32_t x = X, y = Y;
    X = addmod(x, y);
    Y = shoup(submod(x, y), w, ws);
  }
  __device__ __forceinline__ void gs_scaled(uint32_t &X, uint32_t &Y, uint32_t f, uint32_t fs,
                                            uint32_t wf, uint32_t wfs) const {
    const uint32_t x = X, y = Y;
    X = shoup(addmod(x, y), f, fs);
    Y = shoup(submod(x, y), wf, wfs);
  }
  // Montgomery a b 2^-32 mod q, canonical in and out
  __device__ __forceinline__ uint32_t mont(uint32_t a, uint32_t b) const {
    const uint64_t p = (uint64_t)a * b;
    return redc(p, (uint32_t)p * qinv_neg);
  }
  __device__ __forceinline__ uint32_t canon(uint32_t x) const { return x; }
  __device__ __forceinline__ uint32_t canon_inv(uint32_t x) const { return x; }
  static constexpr int kBaseD = 0;  // sums of two canonical products already exceed 2^64
  template <int B, bool NEG, bool ZC = false>
  __device__ void basemul(uint32_t (&)[B], const uint32_t (&)[B], uint32_t, uint32_t) const {}
};

// 64-bit arithmetic on a 32-bit VALU.  q < 2^62 leaves two bits of headroom, so butterflies use
// Harvey's lazy bounds (values in [0, 4q), one conditional subtraction per butterfly instead of
// two), and the Shoup high product is spelled out in 32-bit limbs so hipcc emits v_mad_u64_u32 /
// v_mul_hi_u32 / v_mul_lo_u32 directly (tools/kbench A/B: NTTMUL_A64_PLAIN=1 restores the
// generic __umul64hi / [0, 2q) form).
#ifndef NTTMUL_A64_PLAIN
#define NTTMUL_A64_PLAIN 0
#endif
// borrow-chain csub and mov-lean high product (tools/kbench A/B)
#ifndef NTTMUL_A64_V2
#define NTTMUL_A64_V2 1
#endif
// base multiplication sums from 31-bit limb products (Arith64::basemul): -3.6 % VALU in the C5
// row pass (the 128-bit carries and moves go; the 16 multiply-adds per output stay).  C5 time
// unchanged at the power cap in round 2 (profiles/r2/c5_limb_ab.txt), +0.5 % in round 5
// (profiles/r5/c5_limb/); on round 6's buffer-addressed row pass -0.45 % and -0.36 % in two
// kbench sessions (profiles/r6/ab_c5_limb*.json, identical checksums, same board power): on
#ifndef NTTMUL_A64_LIMB
#define NTTMUL_A64_LIMB 1
#endif
// high product through the carry-out of v_mad_u64_u32 (Arith64::mulhi64; tools/kbench A/B)
#ifndef NTTMUL_A64_MADC
#define NTTMUL_A64_MADC 1
#endif
// inverse outputs canonicalised by one conditional subtraction (Arith64::canon_inv; tools/kbench
// A/B: 0 restores canon's two)
#ifndef NTTMUL_A64_CANON_INV
#define NTTMUL_A64_CANON_INV 1
#endif
// CT sum output through the Shoup product's addend (Arith64::ct; tools/kbench A/B)
#ifndef NTTMUL_A64_ACC
#define NTTMUL_A64_ACC 1
#endif
struct Arith64 {
  using word = uint64_t;
  static constexpr int kBits = 64;
  static constexpr bool kTyped = false;
  static constexpr bool kInvCanonical = false;
  uint64_t q;
  uint64_t qinv_neg;  // -q^-1 mod 2^64
  uint64_t q2;        // 2q, set by the host: opaque to the compiler, so 2x + q2 stays one
                      // v_lshl_add_u64 (from 2q it folds 2x + 2q into 2 (x + q), two instructions)

  // x in [0, 2m) -> [0, m).  Spelled as a 32-bit borrow chain so the select uses the borrow of
  // v_subb_co_u32 directly (the 64-bit __builtin_sub_overflow form adds a v_cmp_gt_u64).
  __device__ __forceinline__ static uint64_t csub(uint64_t x, uint64_t m) {
#if NTTMUL_A64_V2
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    const uint32_t ml = (uint32_t)m, mh = (uint32_t)(m >> 32);
    uint32_t lo, t, hi;
    const bool b1 = __builtin_sub_overflow(xl, ml, &lo);
    const bool b2 = __builtin_sub_overflow(xh, mh, &t);
    const bool b3 = __builtin_sub_overflow(t, (uint32_t)b1, &hi);
    return (b2 | b3) ? x : (((uint64_t)hi << 32) | lo);
#else
    uint64_t d;
    return __builtin_sub_overflow(x, m, &d) ? x : d;
#endif
  }
  // high 64 bits of the 128-bit product x * s, from four 32x32 products.  MADC: the carry-out
  // form below (the butterflies' Shoup products only: in the base multiplication's loops the asm
  // blocks cost the full unroll, and the row kernel fell back to scratch-indexed arrays)
  template <bool MADC = false>
  __device__ __forceinline__ static uint64_t mulhi64(uint64_t x, uint64_t s) {
#if NTTMUL_A64_PLAIN
    return __umul64hi(x, s);
#else
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    const uint32_t sl = (uint32_t)s, sh = (uint32_t)(s >> 32);
#if NTTMUL_A64_MADC
    if constexpr (MADC) {
    // x s = xh sh 2^64 + (xh sl + t) 2^32 + lo32(xl sl) with t = xl sh + hi32(xl sl) < 2^64.
    // xh sl + t can reach 2^65: the carry-out of v_mad_u64_u32 (its SGPR-pair destination, which
    // the compiler's own multiply-adds leave dead) supplies bit 64, so the high product is
    // xh sh + (carry 2^32 + hi32(u)) with no zero-extension moves: 6 VALU instead of 8.
    // s_nop 1: two wait states between the VALU write of the carry mask and its VALU read
    // (the hazard the compiler covers for its own carry chains; it does not see inside asm).
    const uint64_t t = (uint64_t)xl * sh + __umulhi(xl, sl);
    uint64_t u, cc;
    uint32_t c;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %5\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %1, 0, 1, %2"
        : "=&v"(u), "=v"(c), "=&s"(cc)
        : "v"(xh), "v"(sl), "v"(t));
    return (uint64_t)xh * sh + ((u >> 32) | ((uint64_t)c << 32));
    }
#endif
#if NTTMUL_A64_V2
    const uint64_t p00 = (uint64_t)xl * sl;
    const uint64_t t = (uint64_t)xl * sh + (p00 >> 32);
    const uint64_t u = (uint64_t)xh * sl + (t & 0xFFFFFFFFull);
    return (uint64_t)xh * sh + (t >> 32) + (u >> 32);
#else
    const uint64_t t = (uint64_t)xl * sh + __umulhi(xl, sl);
    const uint64_t u = (uint64_t)xh * sl + (uint32_t)t;
    return (uint64_t)xh * sh + ((t >> 32) + (u >> 32));
#endif
#endif
  }
  // low 64 bits of x * w
  __device__ __forceinline__ static uint64_t mullo64(uint64_t x, uint64_t w) {
#if NTTMUL_A64_PLAIN
    return x * w;
#else
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    const uint32_t wl = (uint32_t)w, wh = (uint32_t)(w >> 32);
    const uint64_t a = (uint64_t)xl * wl;
    const uint32_t hi = (uint32_t)(a >> 32) + xl * wh + xh * wl;
    return ((uint64_t)hi << 32) | (uint32_t)a;
#endif
  }
  // acc + (x * w mod q, in [0, 2q)) mod 2^64 for any 64-bit x (Shoup, w' = floor(w 2^64 / q)).
  // The addend rides in the 64-bit addend of the first v_mad_u64_u32 (a constant 0 otherwise), so
  // a Harvey CT gets its sum output x + t without an add of its own (NTTMUL_A64_ACC).
  template <bool MADC = true>
  __device__ __forceinline__ uint64_t shoup(uint64_t x, uint64_t w, uint64_t ws,
                                            uint64_t acc = 0) const {
    const uint64_t qh = mulhi64<MADC>(x, ws);
#if NTTMUL_A64_V2
    // lo64(x w) - lo64(qh q) in one pass: D = xl wl + hl (2^32 - ql) carries the low word and a
    // high word off by +hl, which the complemented constants absorb (2 v_mad_u64_u32,
    // 4 v_mul_lo_u32, 2 v_add3_u32; no 64-bit subtract chain).  Everything is mod 2^64, so acc
    // can join the low sum.
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    const uint32_t wl = (uint32_t)w, wh = (uint32_t)(w >> 32);
    const uint32_t hl = (uint32_t)qh, hh = (uint32_t)(qh >> 32);
    const uint32_t nql = 0u - (uint32_t)q, nqh1 = ~(uint32_t)(q >> 32);
    const uint64_t D = (uint64_t)xl * wl + acc + (uint64_t)hl * nql;
    const uint32_t hi = (uint32_t)(D >> 32) + xl * wh + xh * wl + hl * nqh1 + hh * nql;
    return ((uint64_t)hi << 32) | (uint32_t)D;
#else
    return acc + mullo64(x, w) - mullo64(qh, q);
#endif
  }
#if NTTMUL_A64_PLAIN
  static constexpr uint64_t kLazy = 2;  // values in [0, 2q)
  template <bool XC = false>
  __device__ __forceinline__ void ct(uint64_t &X, uint64_t &Y, uint64_t w, uint64_t ws) const {
    uint64_t x = XC ? X : csub(X, q);
    uint64_t t = csub(shoup(Y, w, ws), q);
    X = x + t;
    Y = x - t + q;
  }
  __device__ __forceinline__ void gs(uint64_t &X, uint64_t &Y, uint64_t w, uint64_t ws) const {
    uint64_t x = csub(X, q), y = csub(Y, q);
    X = x + y;
    Y = shoup(x - y + q, w, ws);
  }
  __device__ __forceinline__ void gs_scaled(uint64_t &X, uint64_t &Y, uint64_t f, uint64_t fs,
                                            uint64_t wf, uint64_t wfs) const {
    uint64_t x = csub(X, q), y = csub(Y, q);
    X = shoup(x + y, f, fs);
    Y = shoup(x - y + q, wf, wfs);
  }
  __device__ __forceinline__ uint64_t canon(uint64_t x) const { return csub(x, q); }
  __device__ __forceinline__ uint64_t canon_inv(uint64_t x) const { return csub(x, q); }
#else
  static constexpr uint64_t kLazy = 4;  // forward values in [0, 4q), inverse values in [0, 2q)
  // Harvey CT: X in [0, 4q), any Y -> outputs in [0, 4q).  NTTMUL_A64_ACC: the sum comes out of
  // the Shoup product's addend and the difference is 2x + 2q - (x + t) (one v_lshl_add_u64 and a
  // 64-bit subtract), one VALU instruction less than x + t and (x + 2q) - t.
  template <bool XC = false>
  __device__ __forceinline__ void ct(uint64_t &X, uint64_t &Y, uint64_t w, uint64_t ws) const {
    const uint64_t x = XC ? X : csub(X, 2 * q);
#if NTTMUL_A64_ACC
    const uint64_t s = shoup(Y, w, ws, x);
    X = s;
    Y = (x << 1) + q2 - s;
#else
    const uint64_t t = shoup(Y, w, ws);
    X = x + t;
    Y = x - t + 2 * q;
#endif
  }
  // Harvey GS: X, Y in [0, 2q) -> outputs in [0, 2q)
  __device__ __forceinline__ void gs(uint64_t &X, uint64_t &Y, uint64_t w, uint64_t ws) const {
    const uint64_t x = X, y = Y;
    X = csub(x + y, 2 * q);
    Y = shoup(x - y + 2 * q, w, ws);
  }
  __device__ __forceinline__ void gs_scaled(uint64_t &X, uint64_t &Y, uint64_t f, uint64_t fs,
                                            uint64_t wf, uint64_t wfs) const {
    const uint64_t x = X, y = Y;
    X = shoup(x + y, f, fs);
    Y = shoup(x - y + 2 * q, wf, wfs);
  }
  // [0, 4q) -> [0, q)
  __device__ __forceinline__ uint64_t canon(uint64_t x) const { return csub(csub(x, 2 * q), q); }
  // [0, 2q) -> [0, q): every value an inverse transform outputs, and every Montgomery product, is
  // below 2q (GS: csub(x + y, 2q) and Shoup products of x, y < 2q; base multiplication and mont:
  // (S + m q) / 2^64 < 2q), so one conditional subtraction canonicalises it where canon's two
  // (for the forward transform's [0, 4q)) were spent before round 6
  __device__ __forceinline__ uint64_t canon_inv(uint64_t x) const {
    return NTTMUL_A64_CANON_INV ? csub(x, q) : canon(x);
  }
#endif
  // Montgomery a b 2^-64 mod q; a, b lazy (< kLazy q) -> [0, 2q).  q < 2^62.
  __device__ __forceinline__ uint64_t mont(uint64_t a, uint64_t b) const {
    a = canon(a);
    b = canon(b);
    const uint64_t lo = mullo64(a, b), hi = mulhi64(a, b);
    const uint64_t m = mullo64(lo, qinv_neg);
    const uint64_t mlo = mullo64(m, q), mhi = mulhi64(m, q);
    const uint64_t s = lo + mlo;
    return hi + mhi + (s < lo ? 1 : 0);  // (t + m q) / 2^64 < 2q
  }
  // Base multiplication of the incomplete transform (see Arith32T::basemul): a = a b 2^-64 in
  // Z_q[x]/(x^B - z), z = (NEG ? -1 : 1) w, Shoup twiddle (w, w').  a, b, b' = z b canonical,
  // each output a 128-bit sum of B products < B q^2 < 2^126, one Montgomery reduction:
  // (S + m q) / 2^64 < q (4q / 2^64 + 1) < 2q.
#ifndef NTTMUL_A64_BASE
#define NTTMUL_A64_BASE 1
#endif
  static constexpr int kBaseD = NTTMUL_A64_BASE ? 2 : 0;
  template <int B, bool NEG, bool ZC = false>
  __device__ __forceinline__ void basemul(uint64_t (&a)[B], const uint64_t (&b)[B], uint64_t w,
                                          uint64_t ws) const {
    static_assert(B == 4, "B products per 128-bit sum");
    if (NEG) {  // -w in Shoup form: (q - w, floor((q - w) 2^64 / q) = ~w')
      w = q - w;
      ws = ~ws;
    }
    uint64_t ar[B], br[B], bz[B];
#pragma unroll
    for (int i = 0; i < B; i++) {
      ar[i] = canon(a[i]);
      br[i] = canon(b[i]);
    }
#pragma unroll
    for (int i = 1; i < B; i++) bz[i] = csub(shoup<false>(b[i], w, ws), q);
#if NTTMUL_A64_LIMB
    // 31-bit limbs: x = xh 2^31 + xl (x < q < 2^62, so both limbs < 2^31).  Each limb product is
    // below 2^62, so the four products of one output sum in a 64-bit accumulator per limb pair
    // with chained v_mad_u64_u32 and no carries (4 instructions per 64 x 64 product instead of
    // ~15 for the 128-bit product and accumulation); the 128-bit sum is assembled once per output.
    uint32_t al[B], ah[B], bl[B], bh[B], zl[B], zh[B];
#pragma unroll
    for (int i = 0; i < B; i++) {
      al[i] = (uint32_t)ar[i] & 0x7FFFFFFFu, ah[i] = (uint32_t)(ar[i] >> 31);
      bl[i] = (uint32_t)br[i] & 0x7FFFFFFFu, bh[i] = (uint32_t)(br[i] >> 31);
      if (i > 0) zl[i] = (uint32_t)bz[i] & 0x7FFFFFFFu, zh[i] = (uint32_t)(bz[i] >> 31);
    }
#endif
#pragma unroll
    for (int k = 0; k < B; k++) {
#if NTTMUL_A64_LIMB
      uint64_t ll = 0, lh = 0, hl = 0, hh = 0;
#pragma unroll
      for (int i = 0; i < B; i++) {
        const uint32_t yl = i <= k ? bl[k - i] : zl[B + k - i];
        const uint32_t yh = i <= k ? bh[k - i] : zh[B + k - i];
        ll += (uint64_t)al[i] * yl;
        lh += (uint64_t)al[i] * yh;
        hl += (uint64_t)ah[i] * yl;
        hh += (uint64_t)ah[i] * yh;
      }
      const unsigned __int128 s = (unsigned __int128)ll +
                                  (((unsigned __int128)lh + hl) << 31) +
                                  ((unsigned __int128)hh << 62);
#else
      unsigned __int128 s = 0;
#pragma unroll
      for (int i = 0; i < B; i++)
        s += (unsigned __int128)ar[i] * (i <= k ? br[k - i] : bz[B + k - i]);
#endif
      const uint64_t lo = (uint64_t)s, hi = (uint64_t)(s >> 64);
      const uint64_t m = lo * qinv_neg;
      // lo + lo64(m q) = 0 mod 2^64: its carry is (lo != 0)
      a[k] = hi + mulhi64(m, q) + (lo != 0 ? 1 : 0);
    }
  }
};

// Twiddle + Shoup companion, stored interleaved so one load fetches both.
template <class W>
struct TwPair {
  W w, ws;
};

}  // namespace nttmul
