/*
 * time_testing_gpu — the reference's timing harness (NTT_Software/NTT_Software_Evaluations/
 * NTT-256/time_testing256.c:118-252) on the GPU product, through the C ABI only.
 *
 * Same flow: read the two coefficient files (ler_coeficientes, :17-44), keep pristine copies, run
 * ntt256_product4 num_inter = 30 times with CLOCK_MONOTONIC around each call (:175-185; the
 * inputs are reset before every call as the reference does, although the GPU product does not
 * clobber them), print the average and the product in print_array format (:46-64).
 *
 *   time_testing_gpu [coeficientes_a.txt coeficientes_b.txt [iterations [batch]]]
 *
 * With batch > 1 it also times one nttmul_multiply_batch_u32 call over `batch` copies of the
 * pair (host buffers: the PCIe-inclusive rate, the FPGA communicator's timing window).
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "nttmul.h"

#define Q 12289
#define N 256

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
  const char *fa = argc > 1 ? argv[1] : "coeficientes_a.txt";
  const char *fb = argc > 2 ? argv[2] : "coeficientes_b.txt";
  int num_inter = argc > 3 ? atoi(argv[3]) : 30;
  size_t batch = argc > 4 ? (size_t)strtoull(argv[4], 0, 0) : 1;
  int32_t A[N] = {0}, B[N] = {0}, C[N] = {0}, At[N], Bt[N];

  printf("Lendo valores a partir do arquivo txt\n");
  if (nttmul_read_coefficients(fa, A, N) < 0 || nttmul_read_coefficients(fb, B, N) < 0) {
    perror("Erro ao abrir o arquivo para leitura");
    return 1;
  }
  memcpy(At, A, sizeof(A));
  memcpy(Bt, B, sizeof(B));

  ntt256_product4(C, A, B); /* first call creates the device context (table upload) */
  printf("Executando mult ntt256 GS(C, A, B) na GPU...\n\n");
  double sum = 0;
  for (int count = 0; count < num_inter; count++) {
    memcpy(A, At, sizeof(A));
    memcpy(B, Bt, sizeof(B));
    double t0 = now();
    ntt256_product4(C, A, B);
    sum += now() - t0;
  }
  printf("Tempo total medio ntt256 gs (GPU): %.3f ms\n", sum / num_inter * 1000);
  printf("(%.2f us por chamada, %d chamadas)\n", sum / num_inter * 1e6, num_inter);

  if (batch > 1) {
    nttmul_ctx *ctx = NULL;
    nttmul_params p = {N, Q, 1002, 1, 0, 0};
    int st = nttmul_create_ex(&ctx, &p);
    uint32_t *a = malloc(batch * N * 4), *b = malloc(batch * N * 4), *c = malloc(batch * N * 4);
    if (st || !a || !b || !c) {
      fprintf(stderr, "Erro: %s\n", nttmul_strerror(st ? st : NTTMUL_ENOMEM));
      return 1;
    }
    for (size_t i = 0; i < batch; i++) {
      memcpy(a + i * N, At, sizeof(At));
      memcpy(b + i * N, Bt, sizeof(Bt));
    }
    nttmul_multiply_batch_u32(ctx, c, a, b, batch); /* warm: staging buffers */
    double t0 = now();
    st = nttmul_multiply_batch_u32(ctx, c, a, b, batch);
    double t = now() - t0;
    if (st || memcmp(c + (batch - 1) * N, C, sizeof(C))) {
      fprintf(stderr, "Erro: batch %s\n", st ? nttmul_strerror(st) : "mismatch");
      return 1;
    }
    printf("Batch %zu (host buffers, PCIe incluso): %.3f ms, %.3f Mpolymults/s\n", batch,
           t * 1000, batch / t / 1e6);
    free(a); free(b); free(c);
    nttmul_destroy(ctx);
  }

  printf("Polinomio C (Resultado C = A * B):\n");
  nttmul_print_array(stdout, C, N);
  printf("\n");
  return 0;
}
