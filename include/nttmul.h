/*
 * nttmul.h — C ABI of the MI355X-native NTT polynomial multiplier (libnttmul.so).
 *
 * Computes c = a * b in Z_q[x]/(x^n + 1) (negacyclic, as the reference's NTT_Software products and
 * colab_programs/schoolbook.py:23-46) with hand-written gfx950 HIP kernels: a psi-merged
 * Cooley-Tukey forward NTT (ntt.C:342-371 mulntt_ct_std2rev), a coefficient-wise modular product
 * (ntt.C:131-137 mul_array) and a psi^-1-merged Gentleman-Sande inverse NTT (ntt.C:428-451
 * nttmul_gs_rev2std), fused per polynomial.  Results are canonical in [0, q) and bit-exact with the
 * reference's ntt256_product1/4 wherever the reference runs, and with its schoolbook definition
 * everywhere else.
 *
 * Replaces, one-for-one:
 *   - Software path: ntt256_product1 / ntt256_product4 (NTT/ntt256.h:270-271) and
 *     ntt_red256_product1 / ntt_red256_product4 (NTT-RED/ntt_red256.h:87,90) — compat shims below.
 *   - FPGA path: Software_Hardware_Comunnicator/linux_app/NTT_PCIECommunicationv2.c:109-252
 *     NTT_HARDWARE_EXE and the Terasic driver it drives (PCIE.c:59-103):
 *       PCIE_Load + PCIE_Open + mode-0 twiddle/param stream  ->  nttmul_create
 *       mode-1 / mode-2 DmaFifoWrite(A, B)                   ->  H2D copies inside nttmul_multiply_*
 *       mode-3 GO + WaitForDoneAll polling                  ->  kernel launch + stream sync
 *       DmaFifoRead(C)                                       ->  D2H copy
 *       szError printf + goto cleanup / return FALSE         ->  negative status + nttmul_strerror
 *       PCIE_Close + PCIE_Unload                             ->  nttmul_destroy
 *
 * Conventions: status 0 = OK, negative = error.  Buffers are caller-owned; the context owns device
 * tables and scratch.  Inputs must be canonical (0 <= x < q); with NTTMUL_FLAG_VALIDATE the library
 * checks them on the device and returns NTTMUL_ERANGE.  New-API inputs are const (never clobbered).
 * A context is used by one host thread at a time; separate contexts are independent.  There is no
 * CPU fallback: without a usable HIP device nttmul_create fails with NTTMUL_ENODEV.
 */
#ifndef NTTMUL_H
#define NTTMUL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NTTMUL_OK 0
#define NTTMUL_EINVAL (-1)       /* bad argument: n not a power of two, q not prime, q != 1 mod 2n */
#define NTTMUL_ENODEV (-2)       /* no HIP device / device index out of range */
#define NTTMUL_EHIP (-3)         /* HIP runtime error (see nttmul_last_error) */
#define NTTMUL_ENOMEM (-4)       /* device or host allocation failed */
#define NTTMUL_ERANGE (-5)       /* an input coefficient was >= q (NTTMUL_FLAG_VALIDATE) */
#define NTTMUL_EUNSUPPORTED (-6) /* (n, q, word) combination outside the implemented kernels */

#define NTTMUL_FLAG_VALIDATE 1u  /* range-check inputs on the device before multiplying */

typedef struct nttmul_ctx nttmul_ctx;

typedef struct {
  uint32_t n;          /* ring degree, power of two, 256 <= n <= 65536                          */
  uint64_t q;          /* prime, q == 1 (mod 2n), q < 2^62                                       */
  uint64_t psi;        /* primitive 2n-th root of unity; 0 = smallest one (generate_params.C:25) */
  int ndev;            /* devices to split host-buffer batches over; <= 0 = all visible devices  */
  int first_dev;       /* first HIP device index used                                           */
  uint32_t flags;      /* NTTMUL_FLAG_*                                                          */
} nttmul_params;

typedef struct {
  uint32_t n, logn;
  uint64_t q, psi, omega, inv_psi, inv_omega, inv_n;
  uint32_t word_bits;  /* 32: lazy 32-bit Shoup kernels (q < 2^31); 64: 64-bit kernels          */
  int ndev;
  int kernel;          /* 1 = fused single-launch polymult, 2 = multi-pass (n > 4096)             */
} nttmul_info;

/* ≙ PCIE_Load + PCIE_Open + mode-0 parameter/twiddle stream (NTT_PCIECommunicationv2.c:137-178) */
int nttmul_create(nttmul_ctx **ctx, uint32_t n, uint64_t q, int ndev);
int nttmul_create_ex(nttmul_ctx **ctx, const nttmul_params *params);
/* ≙ PCIE_Close + PCIE_Unload */
void nttmul_destroy(nttmul_ctx *ctx);

const char *nttmul_strerror(int status);
/* last HIP error string recorded on ctx ("" if none) */
const char *nttmul_last_error(const nttmul_ctx *ctx);
int nttmul_get_info(const nttmul_ctx *ctx, nttmul_info *info);

/* multiply(a, b, n, q) -> c for one polynomial; host buffers of n words.
 * ≙ mode-1 + mode-2 + mode-3 + FIFO read of NTT_HARDWARE_EXE (NTT_PCIECommunicationv2.c:183-224) */
int nttmul_multiply_u32(nttmul_ctx *ctx, uint32_t *c, const uint32_t *a, const uint32_t *b);
int nttmul_multiply_u64(nttmul_ctx *ctx, uint64_t *c, const uint64_t *a, const uint64_t *b);

/* batch of independent products; host buffers [batch][n], row-major.  Split over the context's
 * devices in contiguous slices (no inter-device traffic). */
int nttmul_multiply_batch_u32(nttmul_ctx *ctx, uint32_t *c, const uint32_t *a, const uint32_t *b,
                              size_t batch);
int nttmul_multiply_batch_u64(nttmul_ctx *ctx, uint64_t *c, const uint64_t *a, const uint64_t *b,
                              size_t batch);

/* Device-resident batch on HIP device `dev` (must be one of the context's devices), enqueued on
 * `stream` (a hipStream_t of that device; NULL is the device's null stream, as everywhere in HIP).
 * word_bits = 32 or 64 selects uint32_t or uint64_t coefficient storage.  Asynchronous: returns
 * after the launch; order it with the caller's other work through `stream`. */
int nttmul_multiply_batch_device(nttmul_ctx *ctx, void *c, const void *a, const void *b,
                                 size_t batch, int word_bits, int dev, void *stream);

/* Standalone transforms, so a caller can keep operands in the NTT domain:
 *   forward  = mulntt_ct_std2rev (NTT/ntt.C:342-371; ≙ mul_array16(psi_powers) followed by
 *              ntt_ct_std2rev, the first two steps of ntt256_product1): negacyclic NTT, standard
 *              order in, bit-reversed order out, canonical [0, q).  Equal, element for element,
 *              to the reference's a[] after those two steps.
 *   inverse  = nttmul_gs_rev2std (NTT/ntt.C:428-451) followed by the n^-1 scaling of
 *              ntt256.C:12: bit-reversed in, standard out; inverse(forward(a)) == a.  (The
 *              reference's unscaled inttmul256_gs_rev2std output is n times this.)
 *   pointwise = mul_array (NTT/ntt.C:131-137): c[i] = a[i] * b[i] mod q, canonical.
 * Host-buffer forms take [batch][n] arrays; device forms as nttmul_multiply_batch_device. */
int nttmul_forward_batch_u32(nttmul_ctx *ctx, uint32_t *out, const uint32_t *in, size_t batch);
int nttmul_forward_batch_u64(nttmul_ctx *ctx, uint64_t *out, const uint64_t *in, size_t batch);
int nttmul_inverse_batch_u32(nttmul_ctx *ctx, uint32_t *out, const uint32_t *in, size_t batch);
int nttmul_inverse_batch_u64(nttmul_ctx *ctx, uint64_t *out, const uint64_t *in, size_t batch);
int nttmul_pointwise_batch_u32(nttmul_ctx *ctx, uint32_t *c, const uint32_t *a,
                               const uint32_t *b, size_t batch);
int nttmul_pointwise_batch_u64(nttmul_ctx *ctx, uint64_t *c, const uint64_t *a,
                               const uint64_t *b, size_t batch);
int nttmul_forward_batch_device(nttmul_ctx *ctx, void *out, const void *in, size_t batch,
                                int word_bits, int dev, void *stream);
int nttmul_inverse_batch_device(nttmul_ctx *ctx, void *out, const void *in, size_t batch,
                                int word_bits, int dev, void *stream);
int nttmul_pointwise_batch_device(nttmul_ctx *ctx, void *c, const void *a, const void *b,
                                  size_t batch, int word_bits, int dev, void *stream);

/* Synthetic inputs on the device: a[p][i] = splitmix64(seed + 2n(p0+p) + i) mod q,
 * b[p][i] = splitmix64(seed + 2n(p0+p) + n + i) mod q, for p in [0, count).  Asynchronous. */
int nttmul_fill_random_device(nttmul_ctx *ctx, void *a, void *b, uint64_t p0, size_t count,
                              uint64_t seed, int word_bits, int dev, void *stream);

/* Compat shims with the reference's exact signatures and semantics: n = 256, q = 12289,
 * psi = 1002 (ntt256_tables.h:20-24), int32 coefficients in [0, q-1], result in c.  Like the
 * reference they return nothing; a HIP failure prints the error and aborts (the reference's only
 * failure mode is assert, ntt.C:31 / ntt_red.c:42).  a and b are not modified (the reference uses
 * them as scratch; no caller reads them back, time_testing256.c:110-116 resets them).  The two
 * variants return the same product, as the reference's do. */
void ntt256_product1(int32_t *c, int32_t *a, int32_t *b);
void ntt256_product4(int32_t *c, int32_t *a, int32_t *b);
void ntt_red256_product1(int32_t *c, int32_t *a, int32_t *b);
void ntt_red256_product4(int32_t *c, int32_t *a, int32_t *b);

#ifdef __cplusplus
}
#endif

#endif /* NTTMUL_H */
