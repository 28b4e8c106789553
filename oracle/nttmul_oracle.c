/*
 * nttmul_oracle.c — CPU restatement of the reference's NTT_Software polynomial product.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libnttmul.so, the HIP kernels, the C ABI)
 * links, loads or calls this file.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the reported CPU baseline.
 *
 * What it restates (reference = regras/NTT-based-polynomial-multiplier-FPGA, paths relative to
 * Multiplier_NTT_Based/NTT_Software/NTT_Software_Evaluations/NTT-256/):
 *   - NTT/ntt.C        : the 8 transform loop variants + elementwise products + bitrev shuffle
 *   - NTT/ntt256.C     : ntt256_product1 (CT) and ntt256_product4 (GS) sequences
 *   - NTT/ntt.h:63-183 : the table conventions (generated here for any (n, q, psi))
 *   - NTT-RED/ntt_red.c, ntt_red256.C : the K-RED "optimized" product (q = 12289 only)
 *   - Generator_Params/generate_params.C:25-44 : psi = smallest element of order exactly 2n
 *   - colab_programs/schoolbook.py:23-46       : negacyclic schoolbook (the reference's
 *                                                definition of a correct product)
 * The reference hard-wires Q = 12289 (ntt.C:18) and uint16 tables; this restatement keeps the
 * loop structure exactly and replaces the Q-specialised arithmetic (ntt.C:69-107) by generic
 * modular arithmetic on uint64_t values in [0, q), q < 2^63.
 *
 * Parity pinning: tests/test_oracle.py checks every restated function bit-exactly against the
 * reference compiled from its own sources (oracle/_ref, built by oracle/Makefile) and against
 * tests/golden/ fixtures generated from that build (tests/golden/make_golden.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------------------------ */
/* Modular arithmetic (generic replacement for ntt.C:69-107)                                   */
/* ------------------------------------------------------------------------------------------ */

static inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) {
  return (uint64_t)(((u128)a * b) % q);
}
/* ntt.C:76-81 add_mod: inputs in [0, q-1] */
static inline uint64_t add_mod(uint64_t x, uint64_t y, uint64_t q) {
  uint64_t s = x + y;
  return s >= q ? s - q : s;
}
/* ntt.C:69-74 sub_mod: inputs in [0, q-1] */
static inline uint64_t sub_mod(uint64_t x, uint64_t y, uint64_t q) {
  return x >= y ? x - y : x + (q - y);
}

uint64_t orc_powmod(uint64_t b, uint64_t e, uint64_t q) {
  uint64_t r = 1 % q;
  b %= q;
  while (e) {
    if (e & 1) r = mulmod(r, b, q);
    b = mulmod(b, b, q);
    e >>= 1;
  }
  return r;
}

/* Generator_Params/helper.C:22 modinv (egcd); q is prime here so Fermat gives the same value */
uint64_t orc_invmod(uint64_t a, uint64_t q) { return orc_powmod(a, q - 2, q); }

/* Generator_Params/prime_generate.C:23 miller_rabin — deterministic bases for q < 2^64 */
int orc_is_prime(uint64_t n) {
  static const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2) return 0;
  for (int i = 0; i < 12; i++) {
    if (n == bases[i]) return 1;
    if (n % bases[i] == 0) return 0;
  }
  uint64_t d = n - 1;
  int s = 0;
  while ((d & 1) == 0) { d >>= 1; s++; }
  for (int i = 0; i < 12; i++) {
    uint64_t x = orc_powmod(bases[i], d, n);
    if (x == 1 || x == n - 1) continue;
    int comp = 1;
    for (int r = 1; r < s; r++) {
      x = mulmod(x, x, n);
      if (x == n - 1) { comp = 0; break; }
    }
    if (comp) return 0;
  }
  return 1;
}

/*
 * generate_params.C:25-44: psi = the smallest integer of multiplicative order exactly 2n.
 * The reference scans i = 2, 3, ...; for large q that scan never terminates in practice, so
 * we take any primitive 2n-th root r and return min{ r^k : k odd } — the same set, so the
 * same minimum.  Returns 0 if q is not ≡ 1 (mod 2n).
 */
uint64_t orc_smallest_psi(uint32_t n, uint64_t q) {
  uint64_t two_n = 2ull * n;
  if ((q - 1) % two_n) return 0;
  uint64_t r = 0;
  for (uint64_t g = 2; g < q; g++) {
    uint64_t c = orc_powmod(g, (q - 1) / two_n, q);
    if (orc_powmod(c, n, q) == q - 1) { r = c; break; }
  }
  if (!r) return 0;
  uint64_t r2 = mulmod(r, r, q), best = r, cur = r;
  for (uint64_t k = 3; k < two_n; k += 2) {
    cur = mulmod(cur, r2, q);
    if (cur < best) best = cur;
  }
  return best;
}

/* ------------------------------------------------------------------------------------------ */
/* Tables: the conventions of NTT/ntt.h:63-183 and NTT/ntt256_tables.h, for any (n, q, psi)    */
/* ------------------------------------------------------------------------------------------ */

enum {
  ORC_PSI_POWERS = 0,          /* psi^i                                     */
  ORC_INV_PSI_POWERS,          /* psi^-i                                    */
  ORC_INV_PSI_POWERS_REV,      /* [t+j] = psi^-(n/2t)*bitrev_t(j)           */
  ORC_SCALED_INV_PSI_POWERS,   /* n^-1 psi^-i                               */
  ORC_OMEGA_POWERS,            /* [t+j] = omega^(n/2t)*j                    */
  ORC_OMEGA_POWERS_REV,        /* [t+j] = omega^(n/2t)*bitrev_t(j)          */
  ORC_INV_OMEGA_POWERS,        /* as OMEGA_POWERS with omega^-1             */
  ORC_INV_OMEGA_POWERS_REV,    /* as OMEGA_POWERS_REV with omega^-1         */
  ORC_MIXED_POWERS,            /* [t+j] = psi^(n/2t) omega^(n/2t)*j         */
  ORC_MIXED_POWERS_REV,        /* [t+j] = psi^(n/2t) omega^(n/2t)*bitrev(j) */
  ORC_INV_MIXED_POWERS,        /* as MIXED_POWERS with psi^-1, omega^-1     */
  ORC_INV_MIXED_POWERS_REV,    /* as MIXED_POWERS_REV with psi^-1, omega^-1 */
  ORC_NTAB
};

typedef struct {
  uint32_t n, logn;
  uint64_t q, psi, omega, inv_psi, inv_omega, inv_n;
  uint64_t *tab[ORC_NTAB];
} orc_plan;

static uint32_t bitrev(uint32_t x, uint32_t bits) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < bits; i++) r |= ((x >> i) & 1u) << (bits - 1 - i);
  return r;
}

/* psi == 0 selects orc_smallest_psi(n, q).  Returns NULL on invalid parameters. */
orc_plan *orc_plan_create(uint32_t n, uint64_t q, uint64_t psi) {
  if (n < 2 || (n & (n - 1)) || q < 3 || q >= (1ull << 63)) return NULL;
  if (!psi) psi = orc_smallest_psi(n, q);
  if (!psi || orc_powmod(psi, n, q) != q - 1) return NULL;
  orc_plan *p = (orc_plan *)calloc(1, sizeof(orc_plan));
  p->n = n;
  while ((1u << p->logn) < n) p->logn++;
  p->q = q;
  p->psi = psi;
  p->omega = mulmod(psi, psi, q);
  p->inv_psi = orc_invmod(psi, q);
  p->inv_omega = orc_invmod(p->omega, q);
  p->inv_n = orc_invmod(n % q, q);
  for (int k = 0; k < ORC_NTAB; k++) p->tab[k] = (uint64_t *)calloc(n, sizeof(uint64_t));
  for (uint32_t i = 0; i < n; i++) {
    p->tab[ORC_PSI_POWERS][i] = orc_powmod(psi, i, q);
    p->tab[ORC_INV_PSI_POWERS][i] = orc_powmod(p->inv_psi, i, q);
    p->tab[ORC_SCALED_INV_PSI_POWERS][i] = mulmod(p->inv_n, p->tab[ORC_INV_PSI_POWERS][i], q);
  }
  /* entry 0 is unused by every [t+j] table and is 0 in the reference tables */
  uint32_t lt = 0;
  for (uint32_t t = 1; t < n; t <<= 1, lt++) {
    uint64_t e = n / (2ull * t);
    uint64_t w = orc_powmod(p->omega, e, q), wi = orc_powmod(p->inv_omega, e, q);
    uint64_t ps = orc_powmod(psi, e, q), psi_i = orc_powmod(p->inv_psi, e, q);
    for (uint32_t j = 0; j < t; j++) {
      uint32_t rj = bitrev(j, lt);
      p->tab[ORC_OMEGA_POWERS][t + j] = orc_powmod(w, j, q);
      p->tab[ORC_OMEGA_POWERS_REV][t + j] = orc_powmod(w, rj, q);
      p->tab[ORC_INV_OMEGA_POWERS][t + j] = orc_powmod(wi, j, q);
      p->tab[ORC_INV_OMEGA_POWERS_REV][t + j] = orc_powmod(wi, rj, q);
      p->tab[ORC_MIXED_POWERS][t + j] = mulmod(ps, orc_powmod(w, j, q), q);
      p->tab[ORC_MIXED_POWERS_REV][t + j] = mulmod(ps, orc_powmod(w, rj, q), q);
      p->tab[ORC_INV_MIXED_POWERS][t + j] = mulmod(psi_i, orc_powmod(wi, j, q), q);
      p->tab[ORC_INV_MIXED_POWERS_REV][t + j] = mulmod(psi_i, orc_powmod(wi, rj, q), q);
      p->tab[ORC_INV_PSI_POWERS_REV][t + j] = orc_powmod(p->inv_psi, e * rj, q);
    }
  }
  return p;
}

void orc_plan_destroy(orc_plan *p) {
  if (!p) return;
  for (int k = 0; k < ORC_NTAB; k++) free(p->tab[k]);
  free(p);
}

const uint64_t *orc_plan_table(const orc_plan *p, int which) {
  return (which >= 0 && which < ORC_NTAB) ? p->tab[which] : NULL;
}
void orc_plan_params(const orc_plan *p, uint64_t out[6]) {
  out[0] = p->psi; out[1] = p->omega; out[2] = p->inv_psi;
  out[3] = p->inv_omega; out[4] = p->inv_n; out[5] = p->logn;
}

/* ------------------------------------------------------------------------------------------ */
/* Utilities and elementwise products (ntt.C:27-153)                                           */
/* ------------------------------------------------------------------------------------------ */

/* ntt.C:27-44 */
void orc_bitrev_shuffle(uint64_t *a, uint32_t n) {
  uint32_t i, j, k;
  j = n >> 1;
  for (i = 1; i < n - 1; i++) {
    if (i < j) { uint64_t x = a[i]; a[i] = a[j]; a[j] = x; }
    k = n;
    do { k >>= 1; j ^= k; } while ((j & k) == 0);
  }
}
/* ntt.C:119-125 mul_array16: a[i] = a[i] * p[i] */
void orc_mul_table(uint64_t *a, uint32_t n, const uint64_t *p, uint64_t q) {
  for (uint32_t i = 0; i < n; i++) a[i] = mulmod(a[i], p[i], q);
}
/* ntt.C:131-137 mul_array: c[i] = a[i] * b[i] */
void orc_mul_array(uint64_t *c, uint32_t n, const uint64_t *a, const uint64_t *b, uint64_t q) {
  for (uint32_t i = 0; i < n; i++) c[i] = mulmod(a[i], b[i], q);
}
/* ntt.C:147-153 scalar_mul_array */
void orc_scalar_mul_array(uint64_t *a, uint32_t n, uint64_t c, uint64_t q) {
  for (uint32_t i = 0; i < n; i++) a[i] = mulmod(a[i], c, q);
}

/* ------------------------------------------------------------------------------------------ */
/* The transform loops (ntt.C:168-525), generic modulus                                        */
/* ------------------------------------------------------------------------------------------ */

/* ntt.C:168-197  CT, bit-reversed in, standard out, p[i] = psi^i */
void orc_ntt_ct_rev2std_v1(uint64_t *a, uint32_t n, const uint64_t *p, uint64_t q) {
  uint32_t j, s, t, l;
  for (t = 1, l = n; t < n; t <<= 1, l >>= 1) {
    for (s = 0; s < n; s += t + t) {
      uint64_t x = a[s + t];
      a[s + t] = sub_mod(a[s], x, q);
      a[s] = add_mod(a[s], x, q);
    }
    for (j = 1; j < t; j++) {
      uint64_t w = p[j * l];
      for (s = j; s < n; s += t + t) {
        uint64_t x = mulmod(a[s + t], w, q);
        a[s + t] = sub_mod(a[s], x, q);
        a[s] = add_mod(a[s], x, q);
      }
    }
  }
}

/* ntt.C:216-243  CT, bit-reversed in, standard out, p[t+j] = omega^(n/2t)^j */
void orc_ntt_ct_rev2std(uint64_t *a, uint32_t n, const uint64_t *p, uint64_t q) {
  for (uint32_t t = 1; t < n; t <<= 1) {
    for (uint32_t s = 0; s < n; s += t + t) {
      uint64_t x = a[s + t];
      a[s + t] = sub_mod(a[s], x, q);
      a[s] = add_mod(a[s], x, q);
    }
    for (uint32_t j = 1; j < t; j++) {
      uint64_t w = p[t + j];
      for (uint32_t s = j; s < n; s += t + t) {
        uint64_t x = mulmod(a[s + t], w, q);
        a[s + t] = sub_mod(a[s], x, q);
        a[s] = add_mod(a[s], x, q);
      }
    }
  }
}

/* ntt.C:253-278  psi-merged CT rev2std, p[t+j] = psi^(n/2t) omega^(n/2t)^j */
void orc_mulntt_ct_rev2std(uint64_t *a, uint32_t n, const uint64_t *p, uint64_t q) {
  for (uint32_t t = 1; t < n; t <<= 1) {
    for (uint32_t j = 0; j < t; j++) {
      uint64_t w = p[t + j];
      for (uint32_t s = j; s < n; s += t + t) {
        uint64_t x = mulmod(a[s + t], w, q);
        a[s + t] = sub_mod(a[s], x, q);
        a[s] = add_mod(a[s], x, q);
      }
    }
  }
}

/* ntt.C:295-329  CT, standard in, bit-reversed out, p[t+j] = omega^(n/2t)^bitrev(j) */
void orc_ntt_ct_std2rev(uint64_t *a, uint32_t n, const uint64_t *p, uint64_t q) {
  uint32_t j, s, t, u, d = n;
  for (t = 1; t < n; t <<= 1) {
    d >>= 1;
    for (s = 0; s < d; s++) {
      uint64_t x = a[s + d];
      a[s + d] = sub_mod(a[s], x, q);
      a[s] = add_mod(a[s], x, q);
    }
    u = 0;
    for (j = 1; j < t; j++) {
      uint64_t w = p[t + j];
      u += 2 * d;
      for (s = u; s < u + d; s++) {
        uint64_t x = mulmod(a[s + d], w, q);
        a[s + d] = sub_mod(a[s], x, q);
        a[s] = add_mod(a[s], x, q);
      }
    }
  }
}

/* ntt.C:342-371  psi-merged CT std2rev, p[t+j] = psi^(n/2t) omega^(n/2t)^bitrev(j) */
void orc_mulntt_ct_std2rev(uint64_t *a, uint32_t n, const uint64_t *p, uint64_t q) {
  uint32_t j, s, t, u, d = n;
  for (t = 1; t < n; t <<= 1) {
    d >>= 1;
    for (j = 0, u = 0; j < t; j++, u += 2 * d) {
      uint64_t w = p[t + j];
      for (s = u; s < u + d; s++) {
        uint64_t x = mulmod(a[s + d], w, q);
        a[s + d] = sub_mod(a[s], x, q);
        a[s] = add_mod(a[s], x, q);
      }
    }
  }
}

/* ntt.C:387-416  GS, bit-reversed in, standard out, p[t+j] = omega^(n/2t)^bitrev(j) */
void orc_ntt_gs_rev2std(uint64_t *a, uint32_t n, const uint64_t *p, uint64_t q) {
  uint32_t j, s, t = n, u, d;
  for (d = 1; d < n; d <<= 1) {
    t >>= 1;
    for (s = 0; s < d; s++) {
      uint64_t x = a[s + d];
      a[s + d] = sub_mod(a[s], x, q);
      a[s] = add_mod(a[s], x, q);
    }
    for (j = 1, u = 2 * d; j < t; j++, u += 2 * d) {
      uint64_t w = p[t + j];
      for (s = u; s < u + d; s++) {
        uint64_t x = a[s + d];
        a[s + d] = mulmod(sub_mod(a[s], x, q), w, q);
        a[s] = add_mod(a[s], x, q);
      }
    }
  }
}

/* ntt.C:428-451  psi-merged GS rev2std, p[t+j] = psi^(n/2t) omega^(n/2t)^bitrev(j) */
void orc_nttmul_gs_rev2std(uint64_t *a, uint32_t n, const uint64_t *p, uint64_t q) {
  uint32_t j, s, t = n, u, d;
  for (d = 1; d < n; d <<= 1) {
    t >>= 1;
    for (j = 0, u = 0; j < t; j++, u += 2 * d) {
      uint64_t w = p[t + j];
      for (s = u; s < u + d; s++) {
        uint64_t x = a[s + d];
        a[s + d] = mulmod(sub_mod(a[s], x, q), w, q);
        a[s] = add_mod(a[s], x, q);
      }
    }
  }
}

/* ntt.C:467-493  GS, standard in, bit-reversed out, p[t+j] = omega^(n/2t)^j */
void orc_ntt_gs_std2rev(uint64_t *a, uint32_t n, const uint64_t *p, uint64_t q) {
  for (uint32_t t = n >> 1; t > 0; t >>= 1) {
    for (uint32_t s = 0; s < n; s += t + t) {
      uint64_t x = a[s + t];
      a[s + t] = sub_mod(a[s], x, q);
      a[s] = add_mod(a[s], x, q);
    }
    for (uint32_t j = 1; j < t; j++) {
      uint64_t w = p[t + j];
      for (uint32_t s = j; s < n; s += t + t) {
        uint64_t x = a[s + t];
        a[s + t] = mulmod(sub_mod(a[s], x, q), w, q);
        a[s] = add_mod(a[s], x, q);
      }
    }
  }
}

/* ntt.C:505-525  psi-merged GS std2rev, p[t+j] = psi^(n/2t) omega^(n/2t)^j */
void orc_nttmul_gs_std2rev(uint64_t *a, uint32_t n, const uint64_t *p, uint64_t q) {
  for (uint32_t t = n >> 1; t > 0; t >>= 1) {
    for (uint32_t j = 0; j < t; j++) {
      uint64_t w = p[t + j];
      for (uint32_t s = j; s < n; s += t + t) {
        uint64_t x = a[s + t];
        a[s + t] = mulmod(sub_mod(a[s], x, q), w, q);
        a[s] = add_mod(a[s], x, q);
      }
    }
  }
}

/* ------------------------------------------------------------------------------------------ */
/* Products (NTT/ntt256.C:5-24), generic n                                                    */
/* a and b are clobbered exactly as in the reference (ntt256.h:261-269).                      */
/* ------------------------------------------------------------------------------------------ */

/* ntt256.C:5-13 ntt256_product1 (Cooley-Tukey) */
void orc_product1(const orc_plan *P, uint64_t *c, uint64_t *a, uint64_t *b) {
  uint32_t n = P->n;
  uint64_t q = P->q;
  orc_mul_table(a, n, P->tab[ORC_PSI_POWERS], q);
  orc_ntt_ct_std2rev(a, n, P->tab[ORC_OMEGA_POWERS_REV], q);   /* ntt256.h:37 */
  orc_mul_table(b, n, P->tab[ORC_PSI_POWERS], q);
  orc_ntt_ct_std2rev(b, n, P->tab[ORC_OMEGA_POWERS_REV], q);
  orc_mul_array(c, n, a, b, q);
  orc_ntt_ct_rev2std(c, n, P->tab[ORC_INV_OMEGA_POWERS], q);   /* ntt256.h:45 */
  orc_mul_table(c, n, P->tab[ORC_SCALED_INV_PSI_POWERS], q);
}

/* ntt256.C:16-24 ntt256_product4 (Gentleman-Sande) */
void orc_product4(const orc_plan *P, uint64_t *c, uint64_t *a, uint64_t *b) {
  uint32_t n = P->n;
  uint64_t q = P->q;
  orc_mul_table(a, n, P->tab[ORC_PSI_POWERS], q);
  orc_ntt_gs_std2rev(a, n, P->tab[ORC_OMEGA_POWERS], q);       /* ntt256.h:41 */
  orc_mul_table(b, n, P->tab[ORC_PSI_POWERS], q);
  orc_ntt_gs_std2rev(b, n, P->tab[ORC_OMEGA_POWERS], q);
  orc_mul_array(c, n, a, b, q);
  orc_ntt_gs_rev2std(c, n, P->tab[ORC_INV_OMEGA_POWERS_REV], q); /* ntt256.h:49 */
  orc_mul_table(c, n, P->tab[ORC_SCALED_INV_PSI_POWERS], q);
}

/* psi-merged product: mulntt_ct_std2rev (ntt256.h:58) x2 → mul_array →
 * nttmul_gs_rev2std (ntt256.h:63) → scalar n^-1.  The structure the GPU kernel fuses. */
void orc_product_merged(const orc_plan *P, uint64_t *c, uint64_t *a, uint64_t *b) {
  uint32_t n = P->n;
  uint64_t q = P->q;
  orc_mulntt_ct_std2rev(a, n, P->tab[ORC_MIXED_POWERS_REV], q);
  orc_mulntt_ct_std2rev(b, n, P->tab[ORC_MIXED_POWERS_REV], q);
  orc_mul_array(c, n, a, b, q);
  orc_nttmul_gs_rev2std(c, n, P->tab[ORC_INV_MIXED_POWERS_REV], q);
  orc_scalar_mul_array(c, n, P->inv_n, q);
}

/* colab_programs/schoolbook.py:23-46 negacyclic_multiply: c = a*b in Z_q[x]/(x^n + 1) */
void orc_schoolbook(uint64_t *c, const uint64_t *a, const uint64_t *b, uint32_t n, uint64_t q) {
  for (uint32_t k = 0; k < n; k++) c[k] = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint64_t ai = a[i] % q;
    if (!ai) continue;
    for (uint32_t j = 0; j < n; j++) {
      uint64_t p = mulmod(ai, b[j] % q, q);
      uint32_t k = i + j;
      if (k < n) c[k] = add_mod(c[k], p, q);
      else c[k - n] = sub_mod(c[k - n], p, q);
    }
  }
}

/* Cyclic counterpart, c = a*b mod (x^n - 1, q): what Hardware_Multiplier/PolyMult.v computes
 * (test_generator/helper.py IterativeForwardNTT/IterativeInverseNTT flow, no psi). */
void orc_cyclic_schoolbook(uint64_t *c, const uint64_t *a, const uint64_t *b, uint32_t n,
                           uint64_t q) {
  for (uint32_t k = 0; k < n; k++) c[k] = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint64_t ai = a[i] % q;
    if (!ai) continue;
    for (uint32_t j = 0; j < n; j++) {
      uint32_t k = (i + j) & (n - 1);
      c[k] = add_mod(c[k], mulmod(ai, b[j] % q, q), q);
    }
  }
}

/* Evaluation check: r = psi^(2k+1) is a root of x^n + 1, so
 * c(r) == a(r) b(r) (mod q).  Returns the number of failing points among nk. */
int orc_eval_check(const orc_plan *P, const uint64_t *c, const uint64_t *a, const uint64_t *b,
                   uint32_t nk) {
  uint32_t n = P->n;
  uint64_t q = P->q, r = P->psi, r2 = P->omega;
  int bad = 0;
  for (uint32_t k = 0; k < nk; k++) {
    uint64_t ea = 0, eb = 0, ec = 0;
    for (int32_t i = (int32_t)n - 1; i >= 0; i--) {  /* Horner */
      ea = add_mod(mulmod(ea, r, q), a[i] % q, q);
      eb = add_mod(mulmod(eb, r, q), b[i] % q, q);
      ec = add_mod(mulmod(ec, r, q), c[i] % q, q);
    }
    if (mulmod(ea, eb, q) != ec) bad++;
    r = mulmod(r, r2, q);
  }
  return bad;
}

/* ------------------------------------------------------------------------------------------ */
/* K-RED optimized product, q = 12289 only (NTT-RED/ntt_red.c, NTT-RED/ntt_red256.C)          */
/* Values are signed int32 exactly as in the reference; tables are generated here.            */
/* ------------------------------------------------------------------------------------------ */

#define RQ 12289
static inline int32_t kred(int32_t x) { return 3 * (x & 4095) - (x >> 12); }    /* ntt_red.c:34 */
static inline int32_t kmul_red(int32_t x, int32_t y) {                          /* ntt_red.c:39 */
  int64_t z = (int64_t)x * y;
  return 3 * (int32_t)(z & 4095) - (int32_t)(z >> 12);
}
static void kshift_array(int32_t *a, uint32_t n) {                              /* ntt_red.c:103 */
  for (uint32_t i = 0; i < n; i++) a[i] = (a[i] > (RQ - 1) / 2) ? a[i] - RQ : a[i];
}
static void kreduce_array(int32_t *a, uint32_t n) {                             /* ntt_red.c:124 */
  for (uint32_t i = 0; i < n; i++) a[i] = kred(a[i]);
}
static void kreduce_array_twice(int32_t *a, uint32_t n) {                       /* ntt_red.c:138 */
  for (uint32_t i = 0; i < n; i++) a[i] = kred(kred(a[i]));
}
static void kcorrect(int32_t *a, uint32_t n) {                                  /* ntt_red.c:150 */
  for (uint32_t i = 0; i < n; i++) {
    int32_t x = a[i];
    x += ((x >> 16) & RQ);
    x -= RQ;
    x += ((x >> 16) & RQ);
    a[i] = x;
  }
}
static void kmul_reduce_table(int32_t *a, uint32_t n, const int32_t *p) {       /* ntt_red.c:197 */
  for (uint32_t i = 0; i < n; i++) a[i] = kmul_red(a[i], p[i]);
}
static void kmul_reduce_array(int32_t *c, uint32_t n, const int32_t *a, const int32_t *b) {
  for (uint32_t i = 0; i < n; i++) c[i] = kmul_red(a[i], b[i]);               /* ntt_red.c:205 */
}
static void kntt_ct_rev2std(int32_t *a, uint32_t n, const int32_t *p) {         /* ntt_red.c:244 */
  for (uint32_t t = 1; t < n; t <<= 1) {
    for (uint32_t s = 0; s < n; s += t + t) {
      int32_t x = a[s + t]; a[s + t] = a[s] - x; a[s] = a[s] + x;
    }
    for (uint32_t j = 1; j < t; j++) {
      int32_t w = p[t + j];
      for (uint32_t s = j; s < n; s += t + t) {
        int32_t x = kmul_red(a[s + t], w); a[s + t] = a[s] - x; a[s] = a[s] + x;
      }
    }
  }
}
static void kntt_ct_std2rev(int32_t *a, uint32_t n, const int32_t *p) {         /* ntt_red.c:321 */
  uint32_t d = n;
  for (uint32_t t = 1; t < n; t <<= 1) {
    d >>= 1;
    for (uint32_t s = 0; s < d; s++) {
      int32_t x = a[s + d]; a[s + d] = a[s] - x; a[s] = a[s] + x;
    }
    uint32_t u = 0;
    for (uint32_t j = 1; j < t; j++) {
      int32_t w = p[t + j];
      u += 2 * d;
      for (uint32_t s = u; s < u + d; s++) {
        int32_t x = kmul_red(a[s + d], w); a[s + d] = a[s] - x; a[s] = a[s] + x;
      }
    }
  }
}
static void kntt_gs_rev2std(int32_t *a, uint32_t n, const int32_t *p) {         /* ntt_red.c:414 */
  uint32_t t = n;
  for (uint32_t d = 1; d < n; d <<= 1) {
    t >>= 1;
    for (uint32_t s = 0; s < d; s++) {
      int32_t x = a[s + d]; a[s + d] = a[s] - x; a[s] = a[s] + x;
    }
    uint32_t u = 2 * d;
    for (uint32_t j = 1; j < t; j++, u += 2 * d) {
      int32_t w = p[t + j];
      for (uint32_t s = u; s < u + d; s++) {
        int32_t x = a[s + d]; a[s + d] = kmul_red(a[s] - x, w); a[s] = a[s] + x;
      }
    }
  }
}
static void kntt_gs_std2rev(int32_t *a, uint32_t n, const int32_t *p) {         /* ntt_red.c:495 */
  for (uint32_t t = n >> 1; t > 0; t >>= 1) {
    for (uint32_t s = 0; s < n; s += t + t) {
      int32_t x = a[s + t]; a[s + t] = a[s] - x; a[s] = a[s] + x;
    }
    for (uint32_t j = 1; j < t; j++) {
      int32_t w = p[t + j];
      for (uint32_t s = j; s < n; s += t + t) {
        int32_t x = a[s + t]; a[s + t] = kmul_red(a[s] - x, w); a[s] = a[s] + x;
      }
    }
  }
}

/* centred representative in (-(q-1)/2, (q-1)/2], as the int16 NTT-RED tables store */
static int32_t centre(uint64_t v) { return v > (RQ - 1) / 2 ? (int32_t)v - RQ : (int32_t)v; }

/* K-RED tables (ntt_red256_tables.h conventions): the ntt.h table times 3^-1, centred;
 * scaled inverse psi powers times n^-1 3^-8 (ntt_red256.C:24-25 applies red twice after). */
typedef struct { uint32_t n; int32_t *psi, *omega, *omega_rev, *inv_omega, *inv_omega_rev, *scaled; } kred_tabs;

static void kred_tabs_make(const orc_plan *P, kred_tabs *K) {
  uint32_t n = P->n;
  uint64_t inv3 = orc_invmod(3, RQ), inv3_8 = orc_powmod(inv3, 8, RQ);
  K->n = n;
  K->psi = (int32_t *)malloc(n * 4); K->omega = (int32_t *)malloc(n * 4);
  K->omega_rev = (int32_t *)malloc(n * 4); K->inv_omega = (int32_t *)malloc(n * 4);
  K->inv_omega_rev = (int32_t *)malloc(n * 4); K->scaled = (int32_t *)malloc(n * 4);
  for (uint32_t i = 0; i < n; i++) {
    K->psi[i] = centre(mulmod(P->tab[ORC_PSI_POWERS][i], inv3, RQ));
    K->omega[i] = centre(mulmod(P->tab[ORC_OMEGA_POWERS][i], inv3, RQ));
    K->omega_rev[i] = centre(mulmod(P->tab[ORC_OMEGA_POWERS_REV][i], inv3, RQ));
    K->inv_omega[i] = centre(mulmod(P->tab[ORC_INV_OMEGA_POWERS][i], inv3, RQ));
    K->inv_omega_rev[i] = centre(mulmod(P->tab[ORC_INV_OMEGA_POWERS_REV][i], inv3, RQ));
    K->scaled[i] = centre(mulmod(P->tab[ORC_SCALED_INV_PSI_POWERS][i], inv3_8, RQ));
  }
}
static void kred_tabs_free(kred_tabs *K) {
  free(K->psi); free(K->omega); free(K->omega_rev); free(K->inv_omega); free(K->inv_omega_rev);
  free(K->scaled);
}

/* Exports the generated K-RED tables (centred int32) for the parity test against
 * NTT-RED/ntt_red256_tables.c.  which: 0 psi, 1 omega, 2 omega_rev, 3 inv_omega,
 * 4 inv_omega_rev, 5 scaled_inv_psi. */
int orc_kred_table(const orc_plan *P, int which, int32_t *out) {
  if (P->q != RQ) return -1;
  kred_tabs K;
  kred_tabs_make(P, &K);
  const int32_t *src[6] = {K.psi, K.omega, K.omega_rev, K.inv_omega, K.inv_omega_rev, K.scaled};
  if (which < 0 || which > 5) { kred_tabs_free(&K); return -1; }
  memcpy(out, src[which], P->n * 4);
  kred_tabs_free(&K);
  return 0;
}

/* ntt_red256.C:5-27 (product1, CT) and :30-51 (product4, GS); CT/GS selected by gs.
 * a, b: int32 in [0, q) — clobbered; c: int32 in [0, q).  Returns -1 unless q == 12289. */
int orc_red_product(const orc_plan *P, int gs, int32_t *c, int32_t *a, int32_t *b) {
  if (P->q != RQ) return -1;
  uint32_t n = P->n;
  kred_tabs K;
  kred_tabs_make(P, &K);
  kshift_array(a, n);
  kmul_reduce_table(a, n, K.psi);
  if (gs) kntt_gs_std2rev(a, n, K.omega); else kntt_ct_std2rev(a, n, K.omega_rev);
  kreduce_array(a, n);
  kshift_array(b, n);
  kmul_reduce_table(b, n, K.psi);
  if (gs) kntt_gs_std2rev(b, n, K.omega); else kntt_ct_std2rev(b, n, K.omega_rev);
  kreduce_array(b, n);
  kmul_reduce_array(c, n, a, b);
  kreduce_array_twice(c, n);
  if (gs) kntt_gs_rev2std(c, n, K.inv_omega_rev); else kntt_ct_rev2std(c, n, K.inv_omega);
  kmul_reduce_table(c, n, K.scaled);
  kreduce_array_twice(c, n);
  kcorrect(c, n);
  kred_tabs_free(&K);
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Synthetic inputs: counter-based, so any shard regenerates any polymult        */
/* ------------------------------------------------------------------------------------------ */

static inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* a[p][i] = splitmix64(seed + 2 n (p0+p) + i) mod q ; b[p][i] = ... + n + i */
void orc_fill_inputs(uint64_t *a, uint64_t *b, uint32_t n, uint64_t q, uint64_t seed,
                     uint64_t p0, uint64_t count) {
#pragma omp parallel for schedule(static)
  for (uint64_t p = 0; p < count; p++) {
    uint64_t base = seed + 2ull * n * (p0 + p);
    for (uint32_t i = 0; i < n; i++) {
      a[p * n + i] = splitmix64(base + i) % q;
      b[p * n + i] = splitmix64(base + n + i) % q;
    }
  }
}

/* ------------------------------------------------------------------------------------------ */
/* CPU baseline ("port" of the optimized path): psi-merged, lazy Shoup reduction, u32 words,  */
/* q < 2^31.  Same structure as NTT-RED (merged psi, lazy add/sub, reduce only on twiddle     */
/* products), generalised from K-RED (q = 3*2^12+1 only) to Shoup for any 31-bit prime.       */
/* Batched over OpenMP threads, timed with CLOCK_MONOTONIC like time_testing256.c:178-181.    */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
  uint32_t n, q;
  uint32_t *fw, *fws, *iw, *iws; /* mixed_powers_rev / inv_mixed_powers_rev + Shoup companions */
  uint32_t ninv, ninvs;
  uint64_t mu;                   /* floor(2^64 / q) (Barrett, pointwise product) */
} fast_tabs;

static inline uint32_t shoup32(uint32_t x, uint32_t w, uint32_t ws, uint32_t q) {
  uint32_t qh = (uint32_t)(((uint64_t)x * ws) >> 32);
  return x * w - qh * q; /* in [0, 2q) */
}
static inline uint32_t csub(uint32_t x, uint32_t m) { return x >= m ? x - m : x; }

static void fast_tabs_make(const orc_plan *P, fast_tabs *F) {
  uint32_t n = P->n;
  F->n = n; F->q = (uint32_t)P->q;
  F->fw = (uint32_t *)malloc(n * 4); F->fws = (uint32_t *)malloc(n * 4);
  F->iw = (uint32_t *)malloc(n * 4); F->iws = (uint32_t *)malloc(n * 4);
  for (uint32_t i = 0; i < n; i++) {
    F->fw[i] = (uint32_t)P->tab[ORC_MIXED_POWERS_REV][i];
    F->iw[i] = (uint32_t)P->tab[ORC_INV_MIXED_POWERS_REV][i];
    F->fws[i] = (uint32_t)(((uint64_t)F->fw[i] << 32) / P->q);
    F->iws[i] = (uint32_t)(((uint64_t)F->iw[i] << 32) / P->q);
  }
  F->ninv = (uint32_t)P->inv_n;
  F->ninvs = (uint32_t)(((uint64_t)F->ninv << 32) / P->q);
  F->mu = ~(uint64_t)0 / P->q;
}
static void fast_tabs_free(fast_tabs *F) { free(F->fw); free(F->fws); free(F->iw); free(F->iws); }

/* One CT stage block (ntt.C:365-367 butterfly, lazy [0, 2q)) and one GS stage block
 * (ntt.C:445-447), over d contiguous pairs: restrict-qualified so gcc vectorizes them (AVX2). */
static inline void fast_ct_block(uint32_t *restrict x0, uint32_t *restrict x1, uint32_t d,
                                 uint32_t w, uint32_t ws, uint32_t q) {
  for (uint32_t s = 0; s < d; s++) {
    uint32_t X = csub(x0[s], q), T = csub(shoup32(x1[s], w, ws, q), q);
    x0[s] = X + T;
    x1[s] = X - T + q;
  }
}
static inline void fast_gs_block(uint32_t *restrict x0, uint32_t *restrict x1, uint32_t d,
                                 uint32_t w, uint32_t ws, uint32_t q) {
  for (uint32_t s = 0; s < d; s++) {
    uint32_t X = csub(x0[s], q), Y = csub(x1[s], q);
    x0[s] = X + Y;
    x1[s] = shoup32(X - Y + q, w, ws, q);
  }
}

static void fast_product(const fast_tabs *F, uint32_t *c, const uint32_t *ain, const uint32_t *bin,
                         uint32_t *a, uint32_t *b) {
  uint32_t n = F->n, q = F->q;
  memcpy(a, ain, n * 4);
  memcpy(b, bin, n * 4);
  uint32_t *xs[2] = {a, b};
  for (int k = 0; k < 2; k++) { /* mulntt_ct_std2rev, values kept in [0, 2q) */
    uint32_t *x = xs[k];
    uint32_t d = n;
    for (uint32_t t = 1; t < n; t <<= 1) {
      d >>= 1;
      for (uint32_t j = 0, u = 0; j < t; j++, u += 2 * d)
        fast_ct_block(x + u, x + u + d, d, F->fw[t + j], F->fws[t + j], q);
    }
  }
  /* mul_array (ntt.C:131-137): Barrett with mu = floor(2^64 / q); p < q^2 < 2^62 gives a
   * quotient estimate at most 1 low, so r < 2q < 2^32 */
  const uint64_t mu = F->mu;
  for (uint32_t i = 0; i < n; i++) {
    const uint64_t p = (uint64_t)csub(a[i], q) * csub(b[i], q);
    const uint64_t r = p - (uint64_t)(((u128)p * mu) >> 64) * q;
    c[i] = csub((uint32_t)r, q);
  }
  uint32_t t = n;
  for (uint32_t d = 1; d < n; d <<= 1) { /* nttmul_gs_rev2std */
    t >>= 1;
    for (uint32_t j = 0, u = 0; j < t; j++, u += 2 * d)
      fast_gs_block(c + u, c + u + d, d, F->iw[t + j], F->iws[t + j], q);
  }
  for (uint32_t i = 0; i < n; i++) c[i] = csub(shoup32(c[i], F->ninv, F->ninvs, q), q);
}

/* c, a, b: count polymults, row-major [count][n], uint32 in [0, q).  Returns wall seconds.
 * threads <= 0 uses all OpenMP threads.  Returns -1 if q >= 2^31. */
double orc_fast_batch_u32(const orc_plan *P, uint32_t *c, const uint32_t *a, const uint32_t *b,
                          uint64_t count, int threads) {
  if (P->q >= (1ull << 31)) return -1.0;
  fast_tabs F;
  fast_tabs_make(P, &F);
  uint32_t n = P->n;
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#else
  threads = 1;
#endif
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
#pragma omp parallel num_threads(threads)
  {
    uint32_t *sa = (uint32_t *)malloc(n * 4), *sb = (uint32_t *)malloc(n * 4);
#pragma omp for schedule(static)
    for (int64_t p = 0; p < (int64_t)count; p++)
      fast_product(&F, c + p * n, a + p * n, b + p * n, sa, sb);
    free(sa); free(sb);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  fast_tabs_free(&F);
  return (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
}

/* Batched restated P4 (or P1 with gs=0) on uint64 words, OpenMP over the batch. */
double orc_product_batch(const orc_plan *P, int gs, uint64_t *c, const uint64_t *a,
                         const uint64_t *b, uint64_t count, int threads) {
  uint32_t n = P->n;
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#else
  threads = 1;
#endif
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
#pragma omp parallel num_threads(threads)
  {
    uint64_t *sa = (uint64_t *)malloc(n * 8), *sb = (uint64_t *)malloc(n * 8);
#pragma omp for schedule(static)
    for (int64_t p = 0; p < (int64_t)count; p++) {
      memcpy(sa, a + p * n, n * 8);
      memcpy(sb, b + p * n, n * 8);
      if (gs) orc_product4(P, c + p * n, sa, sb); else orc_product1(P, c + p * n, sa, sb);
    }
    free(sa); free(sb);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
}

/* C1 (BASELINE.json configs[0]): ONE product on ONE core, timed the way time_testing256.c:147-187
 * times ntt256_product4 -- reps iterations, the inputs restored before each (untimed, :110-116),
 * CLOCK_MONOTONIC around the product call only (:178-181), the average returned in seconds.
 * gs = 0: the unoptimized CT sequence (ntt256.C:5-13, orc_product1); 1: GS (ntt256.C:16-24). */
double orc_time_single(const orc_plan *P, int gs, uint64_t *c, const uint64_t *a,
                       const uint64_t *b, int reps) {
  uint32_t n = P->n;
  uint64_t *sa = (uint64_t *)malloc(n * 8), *sb = (uint64_t *)malloc(n * 8);
  double total = 0.0;
  for (int r = 0; r < reps; r++) {
    memcpy(sa, a, n * 8);
    memcpy(sb, b, n * 8);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    if (gs) orc_product4(P, c, sa, sb); else orc_product1(P, c, sa, sb);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    total += (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
  }
  free(sa);
  free(sb);
  return reps > 0 ? total / reps : 0.0;
}

int orc_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
