// ASan/UBSan driver for the host-only code (SURVEY §5 sanitizers): the planner and host API of
// libnttmul (csrc/planner.cpp, csrc/hostapi.cpp — no HIP in either) and the CPU oracle
// (oracle/nttmul_oracle.c, compiled here without OpenMP).  Built and run by
// tests/test_sanitizers.py with -fsanitize=address,undefined -fno-sanitize-recover=all; any
// report aborts the run.  Every check also compares results, so the run is a parity test too.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "nttmul.h"
#include "planner.hpp"

extern "C" {
struct orc_plan;
orc_plan *orc_plan_create(uint32_t n, uint64_t q, uint64_t psi);
void orc_plan_destroy(orc_plan *p);
const uint64_t *orc_plan_table(const orc_plan *p, int which);
uint64_t orc_smallest_psi(uint32_t n, uint64_t q);
int orc_is_prime(uint64_t n);
void orc_product1(const orc_plan *P, uint64_t *c, uint64_t *a, uint64_t *b);
void orc_product4(const orc_plan *P, uint64_t *c, uint64_t *a, uint64_t *b);
void orc_product_merged(const orc_plan *P, uint64_t *c, uint64_t *a, uint64_t *b);
void orc_schoolbook(uint64_t *c, const uint64_t *a, const uint64_t *b, uint32_t n, uint64_t q);
int orc_eval_check(const orc_plan *P, const uint64_t *c, const uint64_t *a, const uint64_t *b,
                   uint32_t points);
void orc_fill_inputs(uint64_t *a, uint64_t *b, uint32_t n, uint64_t q, uint64_t seed,
                     uint64_t p0, uint64_t count);
double orc_fast_batch_u32(const orc_plan *P, uint32_t *c, const uint32_t *a, const uint32_t *b,
                          uint64_t count, int threads);
int orc_red_product(const orc_plan *P, int gs, int32_t *c, int32_t *a, int32_t *b);
}

static int failures = 0;
#define CHECK(cond)                                                         \
  do {                                                                      \
    if (!(cond)) {                                                          \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      failures++;                                                           \
    }                                                                       \
  } while (0)

int main(int argc, char **argv) {
  const char *golden = argc > 1 ? argv[1] : "tests/golden";
  const char *tmp = argc > 2 ? argv[2] : "/tmp";
  struct Case { uint32_t n; uint64_t q; };
  const Case cases[] = {{256, 12289}, {1024, 12289}, {256, 2013265921}, {1024, 1073479681},
                        {4096, 2013265921}, {2048, 4293918721ull},
                        {1024, 0x3FFFFFFFFFE80001ull}};
  for (const Case &cs : cases) {
    const uint32_t n = cs.n;
    const uint64_t q = cs.q;
    CHECK(nttmul_is_prime(q) == orc_is_prime(q));
    const uint64_t psi = nttmul_smallest_psi(n, q);
    CHECK(psi == orc_smallest_psi(n, q));
    orc_plan *P = orc_plan_create(n, q, psi);
    CHECK(P != nullptr);
    std::vector<uint64_t> t(n);
    for (int w = 0; w < 12; w++) {  // the NTT/ntt.h:63-183 tables, planner vs oracle
      CHECK(nttmul_table(n, q, psi, w, t.data()) == NTTMUL_OK);
      CHECK(memcmp(t.data(), orc_plan_table(P, w), n * 8) == 0);
    }
    nttmul::Plan plan;
    CHECK(nttmul::make_plan(n, q, psi, &plan) == NTTMUL_OK);
    CHECK(plan.n == n && plan.q == q && plan.psi == psi && !plan.fw.empty());
    // the restated products against the schoolbook definition (n <= 1024: O(n^2))
    std::vector<uint64_t> a(2 * n), b(2 * n), c1(n), c4(n), cm(n), cs_(n), ta(n), tb(n);
    orc_fill_inputs(a.data(), b.data(), n, q, 0x4E54544D554Cull, 3, 2);
    a[n + 1] = q - 1;
    for (int p = 0; p < 2; p++) {
      uint64_t *ap = &a[p * n], *bp = &b[p * n];
      memcpy(ta.data(), ap, n * 8); memcpy(tb.data(), bp, n * 8);
      orc_product1(P, c1.data(), ta.data(), tb.data());
      memcpy(ta.data(), ap, n * 8); memcpy(tb.data(), bp, n * 8);
      orc_product4(P, c4.data(), ta.data(), tb.data());
      memcpy(ta.data(), ap, n * 8); memcpy(tb.data(), bp, n * 8);
      orc_product_merged(P, cm.data(), ta.data(), tb.data());
      CHECK(c1 == c4 && c4 == cm);
      CHECK(orc_eval_check(P, cm.data(), ap, bp, 4) == 0);
      if (n <= 1024) {
        orc_schoolbook(cs_.data(), ap, bp, n, q);
        CHECK(cs_ == cm);
      }
    }
    if (q < (1ull << 31)) {  // the CPU baseline port (batch of 3, one thread)
      std::vector<uint32_t> a32(3 * n), b32(3 * n), c32(3 * n);
      std::vector<uint64_t> a3(3 * n), b3(3 * n);
      orc_fill_inputs(a3.data(), b3.data(), n, q, 7, 0, 3);
      for (uint32_t i = 0; i < 3 * n; i++) a32[i] = (uint32_t)a3[i], b32[i] = (uint32_t)b3[i];
      CHECK(orc_fast_batch_u32(P, c32.data(), a32.data(), b32.data(), 3, 1) >= 0);
      for (int p = 0; p < 3; p++) {
        orc_product_merged(P, cm.data(), &a3[p * n], &b3[p * n]);
        for (uint32_t i = 0; i < n; i++) CHECK(c32[p * n + i] == cm[i]);
      }
    }
    if (n == 256 && q == 12289) {  // K-RED products (NTT-RED/ntt_red256.C)
      std::vector<int32_t> ra(n), rb(n), rc(n);
      for (int gs = 0; gs < 2; gs++) {
        for (uint32_t i = 0; i < n; i++) ra[i] = (int32_t)a[i], rb[i] = (int32_t)b[i];
        CHECK(orc_red_product(P, gs, rc.data(), ra.data(), rb.data()) == 0);
        orc_product_merged(P, cm.data(), &a[0], &b[0]);
        for (uint32_t i = 0; i < n; i++) CHECK((uint64_t)rc[i] == cm[i]);
      }
    }
    orc_plan_destroy(P);
  }
  // planner edge cases: invalid parameters are refused, not undefined
  nttmul::Plan bad;
  CHECK(nttmul::make_plan(1000, 12289, 0, &bad) != NTTMUL_OK);        // n not a power of two
  CHECK(nttmul::make_plan(256, 12288, 0, &bad) != NTTMUL_OK);         // q not prime
  CHECK(nttmul::make_plan(4096, 12289, 0, &bad) != NTTMUL_OK);        // no 8192-th root
  CHECK(nttmul::make_plan(1u << 17, 0x3FFFFFFFFFE80001ull, 0, &bad) != NTTMUL_OK);  // n too big
  std::vector<uint64_t> t(256);
  CHECK(nttmul_table(256, 12289, 0, 12, t.data()) != NTTMUL_OK);      // table index
  CHECK(nttmul_table(256, 15, 0, 0, t.data()) != NTTMUL_OK);
  uint64_t fq = 0;
  for (int bits = 14; bits <= 62; bits += 8) {
    CHECK(nttmul_find_prime(1024, bits, 0, &fq) == NTTMUL_OK);
    CHECK(fq < (1ull << bits) && fq % 2048 == 1 && nttmul_is_prime(fq));
  }
  CHECK(nttmul_find_prime(1024, 70, 0, &fq) != NTTMUL_OK);
  // FPGA twiddle stream: length query with no buffer, then a capped write
  const size_t len = nttmul_fpga_twiddles(256, 7681, 3844, nttmul_fpga_R(256, 13), 8, nullptr, 0);
  CHECK(len == 272);
  std::vector<uint64_t> w(len + 4, 0xAA);
  CHECK(nttmul_fpga_twiddles(256, 7681, 3844, nttmul_fpga_R(256, 13), 8, w.data(), 10) == len);
  CHECK(w[10] == 0xAA);
  // text formats: the reference's coefficient file, a hex round trip, a missing file
  char path[512];
  snprintf(path, sizeof(path), "%s/coeficientes_a.txt", golden);
  std::vector<int32_t> co(300);
  const int cnt = nttmul_read_coefficients(path, co.data(), 300);
  CHECK(cnt == 256);
  CHECK(nttmul_read_coefficients("/nonexistent/x.txt", co.data(), 4) == -1);
  std::vector<uint64_t> hx(cnt), back(cnt + 8);
  for (int i = 0; i < cnt; i++) hx[i] = (uint64_t)co[i];
  snprintf(path, sizeof(path), "%s/san_hex.txt", tmp);
  CHECK(nttmul_write_hex(path, hx.data(), cnt) >= 0);
  CHECK(nttmul_read_hex(path, back.data(), cnt + 8) == cnt);
  CHECK(memcmp(hx.data(), back.data(), cnt * 8) == 0);
  CHECK(nttmul_read_hex(path, back.data(), 5) == 5);                   // capped read
  FILE *devnull = fopen("/dev/null", "w");
  CHECK(nttmul_print_array(devnull, co.data(), cnt) >= 0);
  fclose(devnull);
  if (failures) {
    fprintf(stderr, "%d checks failed\n", failures);
    return 1;
  }
  printf("sanitizer run ok\n");
  return 0;
}
