// hostapi.cpp — host-only parts of the C ABI: the parameter/twiddle planner API (SURVEY §8f
// row 2), the FPGA-compat twiddle stream (row 3) and the reference's text formats (row 4).
// None of these touch a device.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "nttmul.h"
#include "planner.hpp"

using namespace nttmul;

static uint32_t brev(uint32_t x, uint32_t bits) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < bits; i++) r |= ((x >> i) & 1u) << (bits - 1 - i);
  return r;
}

extern "C" {

int nttmul_is_prime(uint64_t q) { return is_prime(q) ? 1 : 0; }

uint64_t nttmul_smallest_psi(uint32_t n, uint64_t q) {
  if (n < 2 || (n & (n - 1)) || q < 3 || !is_prime(q)) return 0;
  return smallest_psi(n, q);
}

uint64_t nttmul_smallest_omega(uint32_t n, uint64_t q) {
  if (n < 2 || (n & (n - 1)) || q < 3 || !is_prime(q)) return 0;
  return smallest_omega(n, q);
}

int nttmul_find_prime(uint32_t n, int bits, int cyclic, uint64_t *q) {
  if (!q || n < 2 || (n & (n - 1)) || bits < 3 || bits > 62) return NTTMUL_EINVAL;
  const uint64_t m = cyclic ? n : 2ull * n;
  const uint64_t top = (1ull << bits) - 1;
  if (m >= top) return NTTMUL_EINVAL;
  // candidates k m + 1 below 2^bits, from the top down, still of bit length `bits`
  for (uint64_t c = (top - 1) / m * m + 1; c > (1ull << (bits - 1)); c -= m) {
    if (is_prime(c)) {
      *q = c;
      return NTTMUL_OK;
    }
  }
  return NTTMUL_EINVAL;
}

int nttmul_table(uint32_t n, uint64_t q, uint64_t psi, int which, uint64_t *out) {
  if (!out || n < 2 || (n & (n - 1)) || q < 3 || q >= (1ull << 63) || !is_prime(q) ||
      (q - 1) % (2ull * n) || which < 0 || which > 11)
    return NTTMUL_EINVAL;
  if (!psi) psi = smallest_psi(n, q);
  if (!psi || psi >= q || powmod(psi, n, q) != q - 1) return NTTMUL_EINVAL;
  const uint64_t omega = mulmod(psi, psi, q), ipsi = powmod(psi, q - 2, q);
  const uint64_t iomega = mulmod(ipsi, ipsi, q), ninv = powmod(n % q, q - 2, q);
  memset(out, 0, sizeof(uint64_t) * n);
  if (which <= 3 && which != 2) {  // psi_powers, inv_psi_powers, scaled_inv_psi_powers
    const uint64_t base = which == 0 ? psi : ipsi;
    uint64_t v = which == 3 ? ninv : 1;
    for (uint32_t i = 0; i < n; i++) {
      out[i] = v;
      v = mulmod(v, base, q);
    }
    return NTTMUL_OK;
  }
  uint32_t lt = 0;
  for (uint32_t t = 1; t < n; t <<= 1, lt++) {
    const uint64_t e = n / (2ull * t);
    for (uint32_t j = 0; j < t; j++) {
      const uint32_t rj = brev(j, lt);
      uint64_t v;
      switch (which) {
        case 2: v = powmod(ipsi, e * rj, q); break;                 // ntt256_tables.C:84
        case 4: v = powmod(omega, e * j, q); break;                                  // :77-86
        case 5: v = powmod(omega, e * rj, q); break;                                 // :110-114
        case 6: v = powmod(iomega, e * j, q); break;
        case 7: v = powmod(iomega, e * rj, q); break;
        case 8: v = mulmod(powmod(psi, e, q), powmod(omega, e * j, q), q); break;    // :95-97
        case 9: v = mulmod(powmod(psi, e, q), powmod(omega, e * rj, q), q); break;   // :120-122
        case 10: v = mulmod(powmod(ipsi, e, q), powmod(iomega, e * j, q), q); break;
        default: v = mulmod(powmod(ipsi, e, q), powmod(iomega, e * rj, q), q); break;
      }
      out[t + j] = v;
    }
  }
  return NTTMUL_OK;
}

uint64_t nttmul_fpga_R(uint32_t n, int K) {
  int logn = 0;
  while ((1u << logn) < n) logn++;
  const int f = (K + logn) / (logn + 1);  // ceil(K / (logn + 1))
  const int e = (logn + 1) * f;
  return e >= 64 ? 0 : 1ull << e;
}

size_t nttmul_fpga_twiddles(uint32_t n, uint64_t q, uint64_t w, uint64_t R, uint32_t P,
                            uint64_t *out, size_t cap) {
  if (!P || n < 2 || (n & (n - 1)) || !q) return 0;
  const uint32_t PE = 2 * P;
  int logn = 0;
  while ((1u << logn) < n) logn++;
  const uint64_t Rq = R % q;
  size_t idx = 0;
  for (int j = 0; j < logn; j++) {
    const uint32_t lim = ((n / PE) >> j) < 1 ? 1 : ((n / PE) >> j);
    for (uint32_t k = 0; k < lim; k++)
      for (uint32_t i = 0; i < P; i++) {
        const uint64_t wp = (((uint64_t)(P << j) * k + ((uint64_t)i << j)) % (n / 2));
        if (idx < cap && out) out[idx] = mulmod(powmod(w, wp, q), Rq, q);
        idx++;
      }
  }
  return idx;
}

int nttmul_read_coefficients(const char *path, int32_t *out, int max) {
  FILE *f = path ? fopen(path, "r") : nullptr;
  if (!f) return -1;
  int count = 0;
  while (count < max) {
    long long v;
    const int r = fscanf(f, "%lld", &v);
    if (r != 1) break;  // EOF or an invalid token: stop, as ler_coeficientes does
    out[count++] = (int32_t)v;
  }
  fclose(f);
  return count;
}

int nttmul_read_hex(const char *path, uint64_t *out, int max) {
  FILE *f = path ? fopen(path, "r") : nullptr;
  if (!f) return -1;
  char line[256];
  int count = 0;
  while (count < max && fgets(line, sizeof(line), f)) {
    char *p = line;
    while (*p == ' ' || *p == '\t') p++;
    if (p[0] == '/' && p[1] == '/') continue;
    unsigned long long v;
    if (sscanf(p, "%llx", &v) == 1) out[count++] = v;
  }
  fclose(f);
  return count;
}

int nttmul_write_hex(const char *path, const uint64_t *a, int n) {
  FILE *f = path ? fopen(path, "w") : nullptr;
  if (!f) return -1;
  for (int i = 0; i < n; i++) fprintf(f, "%llx\n", (unsigned long long)a[i]);  // hex(x)[2:]
  fclose(f);
  return n;
}

int nttmul_print_array(void *file, const int32_t *a, int n) {
  FILE *f = file ? (FILE *)file : stdout;
  int k = 0;
  for (int i = 0; i < n; i++) {
    if (k == 0) fprintf(f, "  ");
    fprintf(f, "%5d", a[i]);
    k++;
    if (k == 16) {
      fprintf(f, "\n");
      k = 0;
    } else {
      fprintf(f, " ");
    }
  }
  if (k > 0) fprintf(f, "\n");
  return n;
}

}  // extern "C"
