// modarith.hpp — device-side modular arithmetic for the NTT kernels (gfx950).
//
// Replaces the reference's Q=12289-specialised arithmetic (NTT/ntt.C:69-107 add_mod/sub_mod/
// divq/modq; NTT-RED/ntt_red.c:34-46 K-RED) with word-size-generic lazy Shoup butterflies:
//
//   Arith32 : q < 2^31, values kept in [0, 2q) inside 32-bit registers.  A twiddle product is
//             one v_mul_hi_u32 + two v_mul_lo_u32 (Shoup, w' = floor(w 2^32 / q)); a conditional
//             subtraction is v_sub_co_u32 + v_cndmask_b32 (no compare/branch).
//   Arith64 : q < 2^62, values in [0, 2q) in 64-bit registers, 64x64 Shoup via __umul64hi.
//             Also used for 32-bit words with 2^31 <= q < 2^32 (u32 storage, u64 arithmetic).
//
// Pointwise products use Montgomery (R = 2^32 or 2^64); the R^-1 it introduces and the n^-1 of
// the inverse transform are folded into one constant F = n^-1 R (mod q) applied in the last
// inverse stage, so the product needs no separate scaling pass (the reference's final
// mul_array16 by scaled_inv_psi_powers, NTT/ntt256.C:12, disappears into the twiddles).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// conditional-subtract lowering: 0 = e32 sub_co/cndmask asm, 1 = v_min_u32,
// 2 = __builtin_sub_overflow + select (default: measured fastest in k_rows, tools/kbench)
#ifndef NTTMUL_CSUB
#define NTTMUL_CSUB 2
#endif

namespace nttmul {

struct Arith32 {
  using word = uint32_t;
  static constexpr int kBits = 32;
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

  // x * w mod q in [0, 2q) for any 32-bit x (Shoup).
  __device__ __forceinline__ uint32_t shoup(uint32_t x, uint32_t w, uint32_t ws) const {
    uint32_t qh = __umulhi(x, ws);
    return x * w - qh * q;
  }
  // Cooley-Tukey butterfly, ntt.C:365-367 pattern: (X, Y) -> (X + Y w, X - Y w).  In/out [0, 2q).
  __device__ __forceinline__ void ct(uint32_t &X, uint32_t &Y, uint32_t w, uint32_t ws) const {
    uint32_t x = csub(X, q);
    uint32_t t = csub(shoup(Y, w, ws), q);
    X = x + t;
    Y = x - t + q;
  }
  // Gentleman-Sande butterfly, ntt.C:445-447 pattern: (X, Y) -> (X + Y, (X - Y) w).  In/out [0, 2q).
  __device__ __forceinline__ void gs(uint32_t &X, uint32_t &Y, uint32_t w, uint32_t ws) const {
    uint32_t x = csub(X, q), y = csub(Y, q);
    X = x + y;
    Y = shoup(x - y + q, w, ws);
  }
  // Last inverse stage with the output scale F folded in: (X, Y) -> ((X + Y) F, (X - Y) w F).
  __device__ __forceinline__ void gs_scaled(uint32_t &X, uint32_t &Y, uint32_t f, uint32_t fs,
                                            uint32_t wf, uint32_t wfs) const {
    uint32_t x = csub(X, q), y = csub(Y, q);
    X = shoup(x + y, f, fs);
    Y = shoup(x - y + q, wf, wfs);
  }
  // Montgomery product a b 2^-32 mod q, inputs in [0, 2q), output in [0, 2q).
  __device__ __forceinline__ uint32_t mont(uint32_t a, uint32_t b) const {
    uint64_t t = (uint64_t)csub(a, q) * csub(b, q);  // < q^2
    uint32_t m = (uint32_t)t * qinv_neg;
    uint64_t u = t + (uint64_t)m * q;                // < q^2 + 2^32 q < 2^64
    return (uint32_t)(u >> 32);
  }
  __device__ __forceinline__ uint32_t canon(uint32_t x) const { return csub(x, q); }
};

struct Arith64 {
  using word = uint64_t;
  static constexpr int kBits = 64;
  uint64_t q;
  uint64_t qinv_neg;  // -q^-1 mod 2^64

  __device__ __forceinline__ static uint64_t csub(uint64_t x, uint64_t m) {
    uint64_t d;
    return __builtin_sub_overflow(x, m, &d) ? x : d;
  }
  __device__ __forceinline__ uint64_t shoup(uint64_t x, uint64_t w, uint64_t ws) const {
    uint64_t qh = __umul64hi(x, ws);
    return x * w - qh * q;
  }
  __device__ __forceinline__ void ct(uint64_t &X, uint64_t &Y, uint64_t w, uint64_t ws) const {
    uint64_t x = csub(X, q);
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
  // Montgomery a b 2^-64 mod q; a, b in [0, 2q) -> [0, 2q).  q < 2^62.
  __device__ __forceinline__ uint64_t mont(uint64_t a, uint64_t b) const {
    a = csub(a, q);
    b = csub(b, q);
    uint64_t lo = a * b, hi = __umul64hi(a, b);
    uint64_t m = lo * qinv_neg;
    uint64_t mlo = m * q, mhi = __umul64hi(m, q);
    uint64_t s = lo + mlo;
    return hi + mhi + (s < lo ? 1 : 0);  // (t + m q) / 2^64 < 2q
  }
  __device__ __forceinline__ uint64_t canon(uint64_t x) const { return csub(x, q); }
};

// Twiddle + Shoup companion, stored interleaved so one load fetches both.
template <class W>
struct TwPair {
  W w, ws;
};

}  // namespace nttmul
