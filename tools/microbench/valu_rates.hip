// Microbenchmark: VALU issue rate of the instructions a modular butterfly is built from, on gfx950.
// Every op is forced with inline asm (no constant folding), CH independent chains per lane,
// 8 waves per SIMD.  Output: lane-ops/s and cost relative to v_add_u32.  Feeds the VALU roofline
// in DESIGN.md (a Shoup butterfly = 1 mul_hi + 2 mul_lo + ~7 simple ops).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 2048
#define CH 16

#define OP1(ins) asm volatile(ins " %0, %0, %1" : "+v"(v[i]) : "v"(k))
template <int KIND>
__global__ __launch_bounds__(256) void bench(uint32_t *out, uint32_t seed) {
  uint32_t v[CH];
  double d[CH];
  float f[CH];
#pragma unroll
  for (int i = 0; i < CH; i++) {
    v[i] = seed * (threadIdx.x + 1) + i * 0x9E3779B9u;
    d[i] = (double)v[i];
    f[i] = (float)v[i];
  }
  uint32_t k = seed | 1;
  double dk = 1.0000001;
  float fk = 1.0001f;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      if constexpr (KIND == 0) OP1("v_add_u32");
      if constexpr (KIND == 1) OP1("v_mul_lo_u32");
      if constexpr (KIND == 2) OP1("v_mul_hi_u32");
      if constexpr (KIND == 3) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[i]) : "v"(fk));
      if constexpr (KIND == 4) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(dk));
      if constexpr (KIND == 5) OP1("v_mul_u32_u24");
      if constexpr (KIND == 6) OP1("v_min_u32");
      if constexpr (KIND == 7) OP1("v_mul_hi_u32_u24");
      if constexpr (KIND == 8) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(k));
      if constexpr (KIND == 9) {  // v_mad_u64_u32: 64-bit dst
        uint64_t t;
        asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, 0" : "=v"(t) : "v"(v[i]), "v"(k) : "s0", "s1");
        v[i] = (uint32_t)t ^ (uint32_t)(t >> 32);
      }
      if constexpr (KIND == 10) OP1("v_xor_b32");
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < CH; i++) acc ^= v[i] ^ (uint32_t)(int64_t)d[i] ^ (uint32_t)f[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int KIND>
float run(uint32_t *out, int blocks) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  bench<KIND><<<blocks, 256>>>(out, 3);
  (void)hipEventRecord(a);
  for (int r = 0; r < 5; r++) bench<KIND><<<blocks, 256>>>(out, 3 + r);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  int blocks = 256 * 8;
  uint32_t *out; (void)hipMalloc(&out, blocks * 256 * 4);
  const char *names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_fma_f32", "v_fma_f64",
                         "v_mul_u32_u24", "v_min_u32", "v_mul_hi_u32_u24", "v_cndmask_b32",
                         "v_mad_u64_u32+2 (xor,shr)", "v_xor_b32"};
  float ms[11];
  ms[0] = run<0>(out, blocks); ms[1] = run<1>(out, blocks); ms[2] = run<2>(out, blocks);
  ms[3] = run<3>(out, blocks); ms[4] = run<4>(out, blocks); ms[5] = run<5>(out, blocks);
  ms[6] = run<6>(out, blocks); ms[7] = run<7>(out, blocks); ms[8] = run<8>(out, blocks);
  ms[9] = run<9>(out, blocks); ms[10] = run<10>(out, blocks);
  double lane_ops = (double)blocks * 256 * ITERS * CH;
  for (int i = 0; i < 11; i++)
    printf("%-28s %8.3f ms  %8.2f T lane-ops/s  %.2fx v_add_u32\n", names[i], ms[i],
           lane_ops / (ms[i] * 1e-3) / 1e12, ms[i] / ms[0]);
  (void)hipFree(out);
  return 0;
}
