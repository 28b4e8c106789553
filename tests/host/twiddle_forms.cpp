// Host check of the planner's Arith32P twiddle tables (csrc/planner.cpp, arith_select.hpp): every
// forward and inverse entry is the Plantard pair of the reference table value
// (mixed_powers_rev / inv_mixed_powers_rev, nttmul_table), in the form the kernels will use it:
//   - unsigned form: exact for every 32-bit multiplicand (the forward entries at the first stage
//     of a register group, the column passes, the even entries elsewhere);
//   - signed form: exact for every int32 multiplicand in (-q, q) (the odd forward entries of the
//     in-group stages, NTTMUL_P_TYPED 2; the whole inverse table, NTTMUL_P_SIGNED_INV).
// The multiplication is the device sequence restated in 64-bit integer arithmetic.  Built and run
// by tests/test_twiddle_forms.py; prints "twiddle forms ok" and exits 0 on success.
#include <stdint.h>
#include <stdio.h>

#include <random>
#include <vector>

#include "arith_select.hpp"
#include "nttmul.h"
#include "planner.hpp"

static uint32_t pmul(uint32_t x, uint32_t b0, uint32_t b1, uint32_t q) {
  const uint32_t th = (uint32_t)(((uint64_t)x * b0) >> 32) + x * b1;
  return (uint32_t)(((uint64_t)th * q + q) >> 32);
}
static uint32_t pmul_s(int32_t x, uint32_t b0, uint32_t b1s, uint32_t q) {
  const int64_t p = (int64_t)x * (int64_t)(int32_t)b0;            // v_mul_hi_i32
  const uint32_t th = (uint32_t)(p >> 32) + (uint32_t)x * b1s;
  return (uint32_t)(((uint64_t)th * q + (3ull * q + 1) / 2) >> 32);
}
static uint32_t mulmod(uint64_t a, uint64_t b, uint64_t q) {
  return (uint32_t)((unsigned __int128)a * b % q);
}

int main() {
  int bad = 0, checked = 0, signed_fw = 0;
  std::mt19937_64 rng(7);
  const uint32_t ns[] = {256, 1024, 4096, 8192, 65536};
  const uint64_t qs[] = {2013265921ull, 2147352577ull, 1811939329ull};
  for (uint32_t n : ns) {
    for (uint64_t q : qs) {
      if ((q - 1) % (2ull * n)) continue;
      nttmul::Plan P;
      if (nttmul::make_plan(n, q, 0, &P) != 0 || nttmul::a32_kind(q) != nttmul::A32Kind::Plantard) {
        printf("plan failed n=%u q=%llu\n", n, (unsigned long long)q);
        return 1;
      }
      std::vector<uint64_t> fw(n), iw(n);
      if (nttmul_table(n, q, P.psi, 9, fw.data()) || nttmul_table(n, q, P.psi, 11, iw.data())) {
        printf("nttmul_table failed\n");
        return 1;
      }
      for (int dir = 0; dir < 2; dir++) {
        const uint32_t *tab = (const uint32_t *)(dir ? P.iw.data() : P.fw.data());
        const std::vector<uint64_t> &ref = dir ? iw : fw;
        for (uint32_t i = 1; i < n; i++) {
          const bool sgn = dir ? NTTMUL_P_SIGNED_INV
                               : (NTTMUL_P_TYPED >= 2 && nttmul::p_signed_fw_entry((int)P.logn, i));
          signed_fw += !dir && sgn;
          const uint32_t b0 = tab[2 * i], b1 = tab[2 * i + 1], w = (uint32_t)ref[i];
          for (int t = 0; t < 24; t++) {
            if (sgn) {
              const int32_t x = t == 0 ? 0 : t == 1 ? (int32_t)(q - 1) : t == 2 ? -(int32_t)(q - 1)
                                                                   : (int32_t)(rng() % (2 * q - 1)) - (int32_t)(q - 1);
              const uint32_t want = mulmod((uint64_t)((int64_t)x + (int64_t)q), w, q);
              bad += pmul_s(x, b0, b1, (uint32_t)q) != want;
            } else {
              const uint32_t x = t == 0 ? 0u : t == 1 ? 0xFFFFFFFFu : t == 2 ? (uint32_t)(2 * q - 1)
                                                                      : (uint32_t)rng();
              bad += pmul(x, b0, b1, (uint32_t)q) != mulmod(x, w, q);
            }
            checked++;
          }
        }
      }
    }
  }
  // the forward tables must carry signed entries (otherwise the rule silently stopped applying)
  if (NTTMUL_P_TYPED >= 2 && signed_fw == 0) bad++;
  printf("%d products checked, %d signed forward entries, %d wrong\n", checked, signed_fw, bad);
  if (bad) return 1;
  printf("twiddle forms ok\n");
  return 0;
}
