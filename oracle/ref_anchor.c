/* ref_anchor.c — timing anchors on the reference's OWN compiled objects (oracle/_ref/libntt_ref.so,
 * built from /root/reference by oracle/Makefile).  Test/bench infrastructure only: bench.py's
 * cpu_baseline leg reports these beside the port's numbers ("also time the verbatim
 * reference objects at (256, 12289) and (1024, 12289) as anchors").
 *
 * Timing follows NTT-256/time_testing256.c:175-185: restore a and b (the products clobber them,
 * :110-116), CLOCK_MONOTONIC around the product call, average.  The restore is outside the clock.
 * Single thread, like the reference.
 */
#include <stdint.h>
#include <string.h>
#include <time.h>

/* the reference's entry points (NTT/ntt256.h:85-86, NTT-RED/ntt_red256.h:87,90, NTT/ntt.h) */
void ntt256_product1(int32_t *c, int32_t *a, int32_t *b);
void ntt256_product4(int32_t *c, int32_t *a, int32_t *b);
void ntt_red256_product1(int32_t *c, int32_t *a, int32_t *b);
void ntt_red256_product4(int32_t *c, int32_t *a, int32_t *b);
void ntt_ct_std2rev(int32_t *a, uint32_t n, const uint16_t *p);
void ntt_gs_std2rev(int32_t *a, uint32_t n, const uint16_t *p);
void ntt_ct_rev2std(int32_t *a, uint32_t n, const uint16_t *p);
void ntt_gs_rev2std(int32_t *a, uint32_t n, const uint16_t *p);
void mul_array16(int32_t *a, uint32_t n, const uint16_t *p);
void mul_array(int32_t *c, uint32_t n, const int32_t *a, const int32_t *b);

#define NMAX 2048

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

/* which: 0 ntt256_product1, 1 ntt256_product4, 2 ntt_red256_product1, 3 ntt_red256_product4.
 * a0, b0: 256 coefficients in [0, 12289).  Returns seconds per product; c gets the last result. */
double anchor_product256(int which, const int32_t *a0, const int32_t *b0, int32_t *c, int reps) {
  static void (*const fn[4])(int32_t *, int32_t *, int32_t *) = {
      ntt256_product1, ntt256_product4, ntt_red256_product1, ntt_red256_product4};
  if (which < 0 || which > 3 || reps <= 0) return -1.0;
  int32_t a[256], b[256];
  double total = 0.0;
  for (int r = 0; r < reps; r++) {
    memcpy(a, a0, sizeof a);
    memcpy(b, b0, sizeof b);
    const double t0 = now_s();
    fn[which](c, a, b);
    total += now_s() - t0;
  }
  return total / reps;
}

/* The ntt256.C:5-24 sequences driven through the reference's generic-n loops (ntt.C) with
 * caller-generated uint16 tables (the oracle planner's, NTT/ntt.h:63-183 conventions):
 * t[0] psi_powers, t[1] omega_powers, t[2] omega_powers_rev, t[3] inv_omega_powers,
 * t[4] inv_omega_powers_rev, t[5] scaled_inv_psi_powers.  gs: product4 shape, else product1. */
double anchor_product_generic(int gs, uint32_t n, const uint16_t *const t[6], const int32_t *a0,
                              const int32_t *b0, int32_t *c, int reps) {
  if (n > NMAX || reps <= 0) return -1.0;
  int32_t a[NMAX], b[NMAX];
  double total = 0.0;
  for (int r = 0; r < reps; r++) {
    memcpy(a, a0, n * sizeof(int32_t));
    memcpy(b, b0, n * sizeof(int32_t));
    const double t0 = now_s();
    mul_array16(a, n, t[0]);
    mul_array16(b, n, t[0]);
    if (gs) {
      ntt_gs_std2rev(a, n, t[1]);
      ntt_gs_std2rev(b, n, t[1]);
    } else {
      ntt_ct_std2rev(a, n, t[2]);
      ntt_ct_std2rev(b, n, t[2]);
    }
    mul_array(c, n, a, b);
    if (gs)
      ntt_gs_rev2std(c, n, t[4]);
    else
      ntt_ct_rev2std(c, n, t[3]);
    mul_array16(c, n, t[5]);
    total += now_s() - t0;
  }
  return total / reps;
}
