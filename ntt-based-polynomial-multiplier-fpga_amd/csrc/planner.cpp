// planner.cpp — see planner.hpp.
#include "planner.hpp"

#include <string.h>

#include "nttmul.h"

namespace nttmul {

typedef unsigned __int128 u128;

uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)(((u128)a * b) % q); }

uint64_t powmod(uint64_t b, uint64_t e, uint64_t q) {
  uint64_t r = 1 % q;
  b %= q;
  for (; e; e >>= 1) {
    if (e & 1) r = mulmod(r, b, q);
    b = mulmod(b, b, q);
  }
  return r;
}

// prime_generate.C:23 miller_rabin, made deterministic for 64-bit inputs (fixed witness set).
bool is_prime(uint64_t n) {
  static const uint64_t wit[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2) return false;
  for (uint64_t p : wit) {
    if (n == p) return true;
    if (n % p == 0) return false;
  }
  uint64_t d = n - 1;
  int s = 0;
  while (!(d & 1)) { d >>= 1; s++; }
  for (uint64_t a : wit) {
    uint64_t x = powmod(a, d, n);
    if (x == 1 || x == n - 1) continue;
    bool composite = true;
    for (int r = 1; r < s && composite; r++) {
      x = mulmod(x, x, n);
      if (x == n - 1) composite = false;
    }
    if (composite) return false;
  }
  return true;
}

uint64_t smallest_psi(uint32_t n, uint64_t q) {
  const uint64_t two_n = 2ull * n;
  if ((q - 1) % two_n) return 0;
  uint64_t r = 0;
  for (uint64_t g = 2; g < q && !r; g++) {
    uint64_t c = powmod(g, (q - 1) / two_n, q);
    if (powmod(c, n, q) == q - 1) r = c;  // order exactly 2n
  }
  if (!r) return 0;
  // the primitive 2n-th roots are r^k, k odd: take the least
  uint64_t r2 = mulmod(r, r, q), cur = r, best = r;
  for (uint64_t k = 3; k < two_n; k += 2) {
    cur = mulmod(cur, r2, q);
    if (cur < best) best = cur;
  }
  return best;
}

static uint32_t bitrev(uint32_t x, uint32_t bits) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < bits; i++) r |= ((x >> i) & 1u) << (bits - 1 - i);
  return r;
}

static uint64_t companion(uint64_t w, uint64_t q, int bits) {
  return (uint64_t)(((u128)w << bits) / q);
}

// (value, companion) pair the device multiplies by: Shoup (w, floor(w 2^bits / q)); for
// Arith32P (arith_select.hpp) the Plantard constant BR = B q^-1 mod 2^64, B = -w 2^64 mod q, as
// (low, high) words; for the other 32-bit classes the Montgomery form (w 2^32 mod q, that times
// -q^-1 mod 2^32)
// sgn (Arith32P only): the pair for a signed multiplicand x in [-2^31, 2^31) — the high word
// absorbs the sign of the low one (v_mul_hi_i32 reads it as int32): c + (v >> 31)
static void tw_pair(uint64_t w, uint64_t q, int bits, uint64_t *v, uint64_t *c, bool sgn = false) {
  if (bits == 32 && a32_kind(q) == A32Kind::Plantard) {
    uint64_t inv = q;  // q^-1 mod 2^64 (Newton on the 2-adic inverse)
    for (int i = 0; i < 6; i++) inv *= 2 - q * inv;
    const uint64_t r64 = (uint64_t)(((u128)1 << 64) % q);
    const uint64_t b = (q - mulmod(w % q, r64, q)) % q;
    const uint64_t br = b * inv;
    *v = br & 0xFFFFFFFFull;
    *c = br >> 32;
    if (sgn) *c = (*c + (*v >> 31)) & 0xFFFFFFFFull;
    return;
  }
  // Arith32W (q >= 2^31) always takes the Montgomery form
  if (bits == 32 && (NTTMUL_A32_MONT || q >= (1ull << 31))) {
    uint64_t inv = q;
    for (int i = 0; i < 5; i++) inv *= 2 - q * inv;
    const uint64_t w1 = (uint64_t)(((u128)w << 32) % q);
    *v = w1;
    *c = (w1 * (0 - inv)) & 0xFFFFFFFFull;
#if NTTMUL_A32_SEILER
    if (q < (1ull << 31)) *c = (w1 * inv) & 0xFFFFFFFFull;  // Seiler: w1 q^-1 (modarith.hpp)
#endif
    return;
  }
  *v = w;
  *c = companion(w, q, bits);
}

// fw_logn > 0: forward table of an Arith32P plan with NTTMUL_P_TYPED 2: the entries whose
// multiplicand is a signed in-group difference get the signed form (arith_select.hpp)
template <class W>
static void put_pairs(std::vector<uint8_t> &dst, const std::vector<uint64_t> &w, uint64_t q,
                      int bits, bool sgn = false, int fw_logn = 0) {
  dst.assign(w.size() * 2 * sizeof(W), 0);
  W *p = (W *)dst.data();
  for (size_t i = 0; i < w.size(); i++) {
    uint64_t v, c;
    const bool s = sgn || (fw_logn > 0 && NTTMUL_P_TYPED >= 2 && a32_kind(q) == A32Kind::Plantard &&
                           p_signed_fw_entry(fw_logn, (uint32_t)i));
    tw_pair(w[i], q, bits, &v, &c, s);
    p[2 * i] = (W)v;
    p[2 * i + 1] = (W)c;
  }
}

// Centred Montgomery pairs for the N-type operands of modarith.hpp's typed butterflies: after
// the n unsigned pairs (w1 in [0, q)), the same twiddles with w1c = w1 - q when w1 > q / 2, as
// int32 bits, and w2c = w1c (-q^-1) mod 2^32 (= w2 + 1 when shifted).
static void append_centred(std::vector<uint8_t> &dst, uint32_t n, uint64_t q) {
  const size_t half = dst.size();
  dst.resize(2 * half);
  uint32_t *p = (uint32_t *)dst.data();
  uint64_t inv = q;
  for (int i = 0; i < 5; i++) inv *= 2 - q * inv;
  const uint32_t qinv_neg = (uint32_t)(0 - inv);
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t w1 = p[2 * i];
    const uint32_t w1c = w1 > q / 2 ? (uint32_t)(w1 - q) : w1;
    p[2 * n + 2 * i] = w1c;
    p[2 * n + 2 * i + 1] = w1c * qinv_neg;
  }
}

uint64_t smallest_omega(uint32_t n, uint64_t q) {
  if ((q - 1) % n) return 0;
  uint64_t r = 0;
  for (uint64_t g = 2; g < q && !r; g++) {
    uint64_t c = powmod(g, (q - 1) / n, q);
    if (powmod(c, n / 2, q) == q - 1) r = c;  // order exactly n
  }
  if (!r) return 0;
  uint64_t best = r, cur = r;
  for (uint64_t k = 2; k < n; k++) {          // primitive n-th roots: r^k, k odd
    cur = mulmod(cur, r, q);
    if ((k & 1) && cur < best) best = cur;
  }
  return best;
}

int make_plan(uint32_t n, uint64_t q, uint64_t psi, Plan *P, bool cyclic) {
  if (n < 256 || n > 65536 || (n & (n - 1))) return NTTMUL_EINVAL;
  const uint64_t order = cyclic ? n : 2ull * n;
  if (q < 3 || q >= (1ull << 62) || !is_prime(q) || (q - 1) % order) return NTTMUL_EINVAL;
  if (cyclic) {
    // FPGA-compat cyclic convolution (Hardware_Multiplier/PolyMult.v; test_generator/helper.py
    // IterativeForwardNTT): `psi` carries the primitive n-th root omega, no psi weighting.
    if (!psi) psi = smallest_omega(n, q);
    if (!psi || psi >= q || powmod(psi, n / 2, q) != q - 1) return NTTMUL_EINVAL;
  } else {
    if (!psi) psi = smallest_psi(n, q);
    if (!psi || psi >= q || powmod(psi, n, q) != q - 1) return NTTMUL_EINVAL;
  }
  P->cyclic = cyclic;
  P->n = n;
  P->logn = 0;
  while ((1u << P->logn) < n) P->logn++;
  P->q = q;
  P->psi = cyclic ? 0 : psi;
  P->omega = cyclic ? psi : mulmod(psi, psi, q);
  P->inv_psi = cyclic ? 0 : powmod(psi, q - 2, q);
  P->inv_omega = powmod(P->omega, q - 2, q);
  P->inv_n = powmod(n, q - 2, q);
  P->word_bits = q < (1ull << 32) ? 32 : 64;  // 32: Arith32H / Arith32 / Arith32W by q
  const int bits = P->word_bits;

  std::vector<uint64_t> fw(n, 0), iw(n, 0);
  uint32_t lt = 0;
  if (!cyclic) {
    // psi^k, k in [0, 2n): every twiddle is a power of psi (psi^(2n) = 1)
    const uint32_t two_n = 2 * n;
    std::vector<uint64_t> pw(two_n);
    pw[0] = 1;
    for (uint32_t k = 1; k < two_n; k++) pw[k] = mulmod(pw[k - 1], psi, q);
    // mixed_powers_rev[t+j] = psi^(n/2t) omega^((n/2t) bitrev(j)) = psi^(e (1 + 2 bitrev(j))),
    // inv_mixed_powers_rev = its inverse (ntt.h:120-127, :145-155; ntt256.h:58,63)
    for (uint32_t t = 1; t < n; t <<= 1, lt++) {
      const uint64_t e = n / (2ull * t);
      for (uint32_t j = 0; j < t; j++) {
        const uint64_t ex = (e * (1 + 2ull * bitrev(j, lt))) % two_n;
        fw[t + j] = pw[ex];
        iw[t + j] = pw[(two_n - ex) % two_n];
      }
    }
  } else {
    // omega_powers_rev[t+j] = omega^((n/2t) bitrev(j)) and inv_omega_powers_rev (ntt.h:110-117,
    // :134-143): the reference's plain ntt_ct_std2rev / ntt_gs_rev2std tables (ntt256.h:37,49)
    std::vector<uint64_t> pw(n);
    pw[0] = 1;
    for (uint32_t k = 1; k < n; k++) pw[k] = mulmod(pw[k - 1], P->omega, q);
    for (uint32_t t = 1; t < n; t <<= 1, lt++) {
      const uint64_t e = n / (2ull * t);
      for (uint32_t j = 0; j < t; j++) {
        const uint64_t ex = (e * bitrev(j, lt)) % n;
        fw[t + j] = pw[ex];
        iw[t + j] = pw[(n - ex) % n];
      }
    }
  }
  if (bits == 32) {
    put_pairs<uint32_t>(P->fw, fw, q, 32, false, (int)P->logn);
    put_pairs<uint32_t>(P->iw, iw, q, 32, NTTMUL_P_SIGNED_INV);  // GS multiplicands: differences
    if (NTTMUL_A32_MONT && a32_kind(q) == A32Kind::Mont) {  // typed butterflies: centred copies
      append_centred(P->fw, n, q);
      append_centred(P->iw, n, q);
    }
  } else {
    put_pairs<uint64_t>(P->fw, fw, q, 64);
    put_pairs<uint64_t>(P->iw, iw, q, 64);
  }
  // Montgomery constant -q^-1 mod 2^bits (Newton on 2-adic inverse)
  uint64_t inv = q;
  for (int i = 0; i < 6; i++) inv *= 2 - q * inv;
  P->qinv_neg = (0 - inv) & (bits == 32 ? 0xFFFFFFFFull : ~0ull);
  // F = n^-1 R mod q, R = 2^bits: cancels the Montgomery R^-1 of the pointwise product and the
  // n of the unnormalised inverse transform (ntt256.C:12 scaled_inv_psi_powers' n^-1).
  const uint64_t r_mod_q = (uint64_t)(((u128)1 << bits) % q);
  const uint64_t f = mulmod(P->inv_n, r_mod_q, q);
  tw_pair(f, q, bits, &P->f, &P->fs);
  tw_pair(mulmod(iw[1], f, q), q, bits, &P->wf, &P->wfs, NTTMUL_P_SIGNED_INV);
  const uint64_t f4 = mulmod(f, 4, q);
  tw_pair(f4, q, bits, &P->f4, &P->f4s);
  tw_pair(mulmod(iw[1], f4, q), q, bits, &P->wf4, &P->wf4s, NTTMUL_P_SIGNED_INV);
  const uint64_t f8 = mulmod(f, 8, q);
  tw_pair(f8, q, bits, &P->f8, &P->f8s);
  tw_pair(mulmod(iw[1], f8, q), q, bits, &P->wf8, &P->wf8s, NTTMUL_P_SIGNED_INV);
  // standalone inverse NTT: plain n^-1 (ntt256.C:12); pointwise product: R^2 mod q
  tw_pair(P->inv_n, q, bits, &P->fi, &P->fis);
  tw_pair(mulmod(iw[1], P->inv_n, q), q, bits, &P->wfi, &P->wfis, NTTMUL_P_SIGNED_INV);
  // the reference's unscaled inverses (intt*, inttmul*: intt(ntt(a)) = n a, ntt256.h:16-17)
  tw_pair(1, q, bits, &P->fu, &P->fus);
  tw_pair(iw[1], q, bits, &P->wfu, &P->wfus, NTTMUL_P_SIGNED_INV);
  P->r2 = mulmod(r_mod_q, r_mod_q, q);
  return NTTMUL_OK;
}

}  // namespace nttmul
