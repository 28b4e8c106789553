// planner.hpp — host-side parameter and twiddle planner.
//
// Runtime replacement for the reference's compile-time tables and generators:
//   NTT/ntt256_tables.C (precomputed n = 256, q = 12289 tables; conventions ntt.h:63-183),
//   Generator_Params/generate_params.C:12-52 (psi search), prime_generate.C:9-200 (modexp,
//   Miller-Rabin), helper.C:5-35 (modular inverse).
// The reference fixes (n, q) at compile time and stores uint16 tables; here any power-of-two
// n <= 65536 and prime q < 2^62 with q == 1 (mod 2n) is planned at nttmul_create time.
#pragma once
#include <stdint.h>

#include <vector>

#include "arith_select.hpp"

// Arith32 twiddle form (see modarith.hpp); host tables and device kernels must agree
#ifndef NTTMUL_A32_MONT
#define NTTMUL_A32_MONT 1
#endif
#ifndef NTTMUL_A32_SEILER  // modarith.hpp: the A/B variant's tables store w1 q^-1 instead
#define NTTMUL_A32_SEILER 0
#endif

namespace nttmul {

uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q);
uint64_t powmod(uint64_t b, uint64_t e, uint64_t q);
bool is_prime(uint64_t n);
// generate_params.C:25-44 rule: the smallest integer of multiplicative order exactly 2n.
uint64_t smallest_psi(uint32_t n, uint64_t q);
// the smallest integer of multiplicative order exactly n (cyclic / FPGA-compat mode)
uint64_t smallest_omega(uint32_t n, uint64_t q);

struct Plan {
  bool cyclic = false;               // x^n - 1 (FPGA-compat) instead of x^n + 1
  uint32_t n = 0, logn = 0;
  uint64_t q = 0, psi = 0, omega = 0, inv_psi = 0, inv_omega = 0, inv_n = 0;
  int word_bits = 0;                 // 32 when q < 2^32 (table words, kernel family), else 64
  uint64_t qinv_neg = 0, f = 0, fs = 0, wf = 0, wfs = 0;
  uint64_t fi = 0, fis = 0, wfi = 0, wfis = 0, r2 = 0;  // standalone inverse / pointwise
  uint64_t fu = 0, fus = 0, wfu = 0, wfus = 0;          // unscaled inverse (F = 1)
  // product with incomplete transforms (kernels.hip base_mult, D = 2): the inverse skips D
  // stages, so it leaves (n / 2^D) c and the scale is F 2^D
  uint64_t f4 = 0, f4s = 0, wf4 = 0, wf4s = 0;
  uint64_t f8 = 0, f8s = 0, wf8 = 0, wf8s = 0;  // D = 3 (Arith32P3)
  // interleaved {w, w'} pairs (u32 or u64 each), n entries; entry 0 unused
  std::vector<uint8_t> fw, iw;
};

// Returns 0 or a negative NTTMUL_E* status.
int make_plan(uint32_t n, uint64_t q, uint64_t psi, Plan *out, bool cyclic = false);

}  // namespace nttmul
