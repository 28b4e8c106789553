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
 *   - Software path: ntt256_product1 / ntt256_product4 (NTT/ntt256.h:85-86) and
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
#define NTTMUL_FLAG_CYCLIC 2u    /* FPGA-compat: c = a*b mod (x^n - 1, q) (Hardware_Multiplier/
                                    PolyMult.v); q == 1 (mod n); params.psi carries omega */
#define NTTMUL_FLAG_SHARE_DEVICES 4u /* params.ndev slices may exceed the visible devices: slice i
                                    runs on device first_dev + i mod (count - first_dev), with its
                                    own streams and buffers (the multi-device split on one GPU) */

typedef struct nttmul_ctx nttmul_ctx;

typedef struct {
  uint32_t n;          /* ring degree, power of two, 256 <= n <= 65536                          */
  uint64_t q;          /* prime, q == 1 (mod 2n), q < 2^62                                       */
  uint64_t psi;        /* primitive 2n-th root of unity; 0 = smallest one (generate_params.C:25) */
  int ndev;            /* devices (slices) to split host-buffer batches over, each driven by its
                          own host thread; <= 0 = all visible devices                           */
  int first_dev;       /* first HIP device index used                                           */
  uint32_t flags;      /* NTTMUL_FLAG_*                                                          */
  /* Dispatch and runtime knobs, read once by nttmul_create_sized (0 = the default in brackets; a
   * zero-initialised struct gets every default; nttmul_create_ex reads the six fields above only
   * and gives these their defaults).  The library reads no environment variable. */
  int32_t issue_prio;   /* fused products (n <= 4096, q < 2^31): 0 = automatic [the issue-
                           prioritised kernel for launches of at most 4 waves per SIMD made on the
                           same stream as the context's previous product launch], 1 = always,
                           -1 = never (oldest-first issue)                                       */
  int32_t zero_copy_kb; /* host-buffer calls, n <= 4096: per-operand chunks up to this many KiB
                           run zero-copy on the pinned staging buffers [64]; -1 = never          */
  int32_t copy_threads; /* host threads splitting each large staging copy [8], capped at the
                           host's hardware threads                                              */
  uint32_t scratch_mb;  /* n > 4096 products and reordered transforms: at most this many MiB per
                           scratch buffer; larger batches run in sub-batches through it [512]   */
  int32_t small_server; /* host-buffer products of at most 1024 words per operand (n <= 1024,
                           q < 2^31, 32-bit words): 0 = served by a resident device kernel
                           that polls a mailbox (go, a, b in device memory the host writes
                           through its BAR mapping, or page-locked host memory without one; c
                           in page-locked host memory), the FPGA's GO / done-all handshake
                           without a launch per call [automatic; the kernel leaves after 1 ms
                           without a request (50 ms in all) and is relaunched on demand; it also
                           leaves before the context enqueues any other work];
                           -1 = a kernel launch per call                                        */
} nttmul_params;
/* Bytes of the round 1-3 nttmul_params (n .. flags): what nttmul_create_ex reads. */
#define NTTMUL_PARAMS_BASE_SIZE offsetof(nttmul_params, issue_prio)

typedef struct {
  uint32_t n, logn;
  uint64_t q, psi, omega, inv_psi, inv_omega, inv_n;
  uint32_t word_bits;  /* 32: 32-bit kernels (q < 2^32); 64: 64-bit kernels (q < 2^62)           */
  int ndev;
  int kernel;          /* 1 = fused single-launch polymult, 2 = multi-pass (n > 4096)             */
  uint32_t cyclic;     /* 1 with NTTMUL_FLAG_CYCLIC (psi, inv_psi are 0 then)                    */
} nttmul_info;

/* ≙ PCIE_Load + PCIE_Open + mode-0 parameter/twiddle stream (NTT_PCIECommunicationv2.c:137-178) */
int nttmul_create(nttmul_ctx **ctx, uint32_t n, uint64_t q, int ndev);
/* the fields n .. flags of *params (NTTMUL_PARAMS_BASE_SIZE bytes); the knobs take defaults.
 * Compatibility note (advisor r5): in round 4 this entry point also read the knob fields
 * (issue_prio .. small_server).  Since round 5 it reads the round 1-3 layout only, so a binary
 * built against the round-4 header that sets those knobs through nttmul_create_ex gets their
 * defaults without an error: such a binary must be rebuilt to call nttmul_create_sized with
 * sizeof(nttmul_params). */
int nttmul_create_ex(nttmul_ctx **ctx, const nttmul_params *params);
/* the first params_size bytes of *params, the rest defaults: pass sizeof(nttmul_params) to set
 * the knobs.  NTTMUL_EINVAL for params_size below NTTMUL_PARAMS_BASE_SIZE or above the size this
 * library knows (fields it could not honour). */
int nttmul_create_sized(nttmul_ctx **ctx, const nttmul_params *params, size_t params_size);
/* ≙ PCIE_Close + PCIE_Unload */
void nttmul_destroy(nttmul_ctx *ctx);

const char *nttmul_strerror(int status);
/* last HIP error string recorded on ctx ("" if none) */
const char *nttmul_last_error(const nttmul_ctx *ctx);
int nttmul_get_info(const nttmul_ctx *ctx, nttmul_info *info);
/* Diagnostics (no reference counterpart): the device kernel(s) one product call with word_bits
 * storage dispatches to, as rocprofv3 names them with template arguments, e.g.
 * "k_rows<Arith32P3,u32,u32,12,0>" (n > 4096: the passes joined by " + ").  Copies at most
 * cap - 1 characters and a NUL into buf; returns the full length, or a negative status.
 * nttmul_kernel_name describes a large batch; nttmul_kernel_name_batch the given one (batches of
 * at most 4 waves per SIMD run the issue-prioritised variant, named "...,prio>"). */
int nttmul_kernel_name(const nttmul_ctx *ctx, int word_bits, char *buf, size_t cap);
int nttmul_kernel_name_batch(const nttmul_ctx *ctx, int word_bits, size_t batch, char *buf,
                             size_t cap);
/* The kernel(s) the context's last product launch ran (same format; "" before the first one):
 * also reflects choices made per call, e.g. the issue-prioritised variant left off when
 * consecutive calls alternate over streams. */
int nttmul_last_kernel_name(const nttmul_ctx *ctx, char *buf, size_t cap);
/* Diagnostics: how the last host-buffer call on ctx moved its first chunk: 0 staged through
 * pinned buffers, 1 direct DMA from / to page-locked caller memory, 2 zero-copy kernel access to
 * the pinned staging buffers, 3 the resident device server's mailbox (params.small_server);
 * -1 before any call. */
int nttmul_last_host_path(const nttmul_ctx *ctx);
/* Diagnostics: setup or launch failures of the context's device server (params.small_server) so
 * far (>= 0; NTTMUL_EINVAL without a context), and the last one's message in reason (cap bytes,
 * "" when none): the call that met the failure ran on the launch path instead, an out-of-memory
 * failure retries the server after 64 more eligible calls (up to 3 failures), any other failure
 * leaves the launch path for the context's lifetime. */
int nttmul_server_status(const nttmul_ctx *ctx, char *reason, size_t cap);

/* multiply(a, b, n, q) -> c for one polynomial; host buffers of n words.
 * ≙ mode-1 + mode-2 + mode-3 + FIFO read of NTT_HARDWARE_EXE (NTT_PCIECommunicationv2.c:183-224) */
int nttmul_multiply_u32(nttmul_ctx *ctx, uint32_t *c, const uint32_t *a, const uint32_t *b);
int nttmul_multiply_u64(nttmul_ctx *ctx, uint64_t *c, const uint64_t *a, const uint64_t *b);

/* batch of independent products; host buffers [batch][n], row-major.  Split over the context's
 * devices in contiguous slices (no inter-device traffic).  Buffers in pageable memory are staged
 * through the context's pinned buffers by host threads (the bound of this path); when a, b and c
 * all lie in page-locked memory (nttmul_host_alloc, or hipHostMalloc / hipHostRegister by the
 * caller) the copy engines DMA the chunks straight from and to them, as the FPGA communicator's
 * PCIE_DmaWrite / PCIE_DmaRead did from its own buffers (NTT_PCIECommunicationv2.c:164-229).
 * batch = 0 is a successful no-op (the pointers may then be NULL; here and on the device path);
 * a NULL operand with batch > 0, or 32-bit words for a q >= 2^32, is NTTMUL_EINVAL. */
int nttmul_multiply_batch_u32(nttmul_ctx *ctx, uint32_t *c, const uint32_t *a, const uint32_t *b,
                              size_t batch);
int nttmul_multiply_batch_u64(nttmul_ctx *ctx, uint64_t *c, const uint64_t *a, const uint64_t *b,
                              size_t batch);

/* Page-locked host memory for the host-buffer calls above (the DMA buffers of the FPGA flow,
 * NTT_PCIECommunicationv2.c:164-229 PCIE_DmaWrite/DmaRead): *p = NULL and NTTMUL_ENOMEM on
 * failure, NTTMUL_ENODEV without a device.  Free with nttmul_host_free. */
int nttmul_host_alloc(void **p, size_t bytes);
void nttmul_host_free(void *p);

/* Device-resident batch on HIP device `dev` (must be one of the context's devices), enqueued on
 * `stream` (a hipStream_t of that device; NULL is the device's null stream, as everywhere in HIP).
 * word_bits = 32 or 64 selects uint32_t or uint64_t coefficient storage.  Asynchronous: returns
 * after the launch; order it with the caller's other work through `stream`.  Calls on different
 * streams may be mixed: for n > 4096 (and the reordered transforms) the context's scratch is
 * handed from one call to the next by a HIP event, so such calls run in enqueue order. */
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

/* General transform entry point: the reference's whole wrapper set (NTT/ntt256.h:20-69) for any
 * context.  mode = direction | order | scaling:
 *   NTTMUL_XF_FORWARD / NTTMUL_XF_INVERSE
 *   NTTMUL_XF_STD2REV : standard-order input, bit-reversed output (ntt_ct/gs_std2rev)
 *   NTTMUL_XF_REV2STD : bit-reversed input, standard-order output (ntt_ct/gs_rev2std)
 *   NTTMUL_XF_UNSCALED: inverse without n^-1, as the reference's intt* / inttmul* (ntt256.h:16-17:
 *                       intt(ntt(a)) = n a)
 * On a negacyclic context the forward is mulntt (psi weights merged, ntt.C:257-371) and the
 * inverse nttmul / inttmul (psi^-1 merged, ntt.C:387-493); on a NTTMUL_FLAG_CYCLIC context they
 * are the plain ntt / intt with omega.  The CT and GS loops of the reference give identical
 * results for the same order, so there is one entry per (direction, order, scaling).
 * nttmul_forward_* == FORWARD | STD2REV, nttmul_inverse_* == INVERSE | REV2STD. */
#define NTTMUL_XF_FORWARD 0u
#define NTTMUL_XF_INVERSE 1u
#define NTTMUL_XF_STD2REV 0u
#define NTTMUL_XF_REV2STD 2u
#define NTTMUL_XF_UNSCALED 4u
int nttmul_transform_batch_u32(nttmul_ctx *ctx, unsigned mode, uint32_t *out, const uint32_t *in,
                               size_t batch);
int nttmul_transform_batch_u64(nttmul_ctx *ctx, unsigned mode, uint64_t *out, const uint64_t *in,
                               size_t batch);
int nttmul_transform_device(nttmul_ctx *ctx, unsigned mode, void *out, const void *in,
                            size_t batch, int word_bits, int dev, void *stream);

/* Synthetic inputs on the device: a[p][i] = splitmix64(seed + 2n(p0+p) + i) mod q,
 * b[p][i] = splitmix64(seed + 2n(p0+p) + n + i) mod q, for p in [0, count).  Asynchronous. */
int nttmul_fill_random_device(nttmul_ctx *ctx, void *a, void *b, uint64_t p0, size_t count,
                              uint64_t seed, int word_bits, int dev, void *stream);

/* ---- Parameter / twiddle planner (host only, no device needed) ----------
 * Replaces Generator_Params/ (generate_params.C:12-73, prime_generate.C:9-200, helper.C:5-35)
 * and the precomputed NTT/ntt256_tables.C with run-time generation for any (n, q, psi). */
int nttmul_is_prime(uint64_t q);                       /* deterministic Miller-Rabin, q < 2^64 */
/* generate_params.C:25-44: the smallest element of multiplicative order exactly 2n (0: none) */
uint64_t nttmul_smallest_psi(uint32_t n, uint64_t q);
/* the smallest element of order exactly n (cyclic mode's omega; 0: none) */
uint64_t nttmul_smallest_omega(uint32_t n, uint64_t q);
/* Largest prime q < 2^bits with q == 1 (mod 2n) (mod n when cyclic), 3 <= bits <= 62: the
 * deterministic counterpart of generate_params.C:16-20's random K-bit search.  0 / NTTMUL_EINVAL */
int nttmul_find_prime(uint32_t n, int bits, int cyclic, uint64_t *q);
/* The tables of NTT/ntt.h:63-183 for (n, q, psi), uint64 in [0, q), n entries; psi = 0 picks
 * nttmul_smallest_psi.  which: 0 psi_powers, 1 inv_psi_powers, 2 inv_psi_powers_rev,
 * 3 scaled_inv_psi_powers, 4 omega_powers, 5 omega_powers_rev, 6 inv_omega_powers,
 * 7 inv_omega_powers_rev, 8 mixed_powers, 9 mixed_powers_rev, 10 inv_mixed_powers,
 * 11 inv_mixed_powers_rev.  For n = 256, q = 12289, psi = 1002 these equal ntt256_tables.C. */
int nttmul_table(uint32_t n, uint64_t q, uint64_t psi, int which, uint64_t *out);

/* ---- FPGA-compat ----------------------------------------------------------
 * R of generate_params.C:47-49: 2^((log2 n + 1) * ceil(K / (log2 n + 1))), K = bits of q */
uint64_t nttmul_fpga_R(uint32_t n, int K);
/* generate_twiddles (generate_params.C:54-73) / test_generator.py:184-189: the PolyMult.v twiddle
 * stream W[idx] = w^((((P << j) k + (i << j)) mod n/2)) R mod q for j < log2 n,
 * k < max(1, (n / 2P) >> j), i < P (P = PE_NUMBER, 8 on the DE2i-150).  Writes at most cap words,
 * returns the stream length (272 for n = 256, P = 8).  Computed in 64-bit (no uint32 overflow). */
size_t nttmul_fpga_twiddles(uint32_t n, uint64_t q, uint64_t w, uint64_t R, uint32_t P,
                            uint64_t *out, size_t cap);

/* ---- Text formats --------------------------------------------------------
 * nttmul_read_coefficients: time_testing256.c:17-44 ler_coeficientes — up to max whitespace-
 * separated decimal int32 values, stopping at EOF or the first invalid token; returns the count
 * read, or -1 if the file cannot be opened.
 * nttmul_read_hex: $readmemh files (test_generator.py:174-181 POLY_*_HEX.txt, NTT_DIN.txt): one
 * hexadecimal word per line, '//' comments skipped; returns the count or -1.
 * nttmul_print_array: time_testing256.c:46-64 print_array — 16 per row, "%5d", two-space indent. */
int nttmul_read_coefficients(const char *path, int32_t *out, int max);
int nttmul_read_hex(const char *path, uint64_t *out, int max);
int nttmul_write_hex(const char *path, const uint64_t *a, int n);
int nttmul_print_array(void *file /* FILE* */, const int32_t *a, int n);

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

/* The reference's n = 256 transform wrappers (NTT/ntt256.h:20-69, there static inline over the
 * ntt.C loops and the ntt256_tables.C tables), in place on int32 a[256] in [0, q-1], same names
 * and results: ntt256_* forward and intt256_* unscaled inverse with omega = psi^2 = 8595
 * (cyclic), mulntt256_* forward with psi merged, inttmul256_* unscaled inverse with psi^-1
 * merged.  A program that included ntt256.h replaces it with this header. */
void ntt256_ct_rev2std(int32_t *a);
void ntt256_gs_rev2std(int32_t *a);
void ntt256_ct_std2rev(int32_t *a);
void ntt256_gs_std2rev(int32_t *a);
void intt256_ct_rev2std(int32_t *a);
void intt256_gs_rev2std(int32_t *a);
void intt256_ct_std2rev(int32_t *a);
void intt256_gs_std2rev(int32_t *a);
void mulntt256_ct_rev2std(int32_t *a);
void mulntt256_ct_std2rev(int32_t *a);
void inttmul256_gs_rev2std(int32_t *a);
void inttmul256_gs_std2rev(int32_t *a);

#ifdef __cplusplus
}
#endif

#endif /* NTTMUL_H */
