// valu_issue — SIMD cycles per wave64 VALU instruction on gfx950, by opcode.
// 2048 blocks x 256 threads (8 waves per SIMD), CH independent chains per lane, inline asm so
// nothing folds.  cycles/instr/SIMD = kernel wall time (hipEvents) x shader clock (s_memtime vs the
// 100 MHz s_memrealtime, measured in-kernel) x 1024 SIMDs / wave-instructions issued.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CH 16
#define ITERS 2048

template <int KIND>
__global__ __launch_bounds__(256) void k(uint64_t *clk, uint32_t *out, uint32_t seed) {
  uint32_t v[CH];
  uint64_t w[CH];
  for (int i = 0; i < CH; i++) v[i] = seed * (threadIdx.x + 1) + i, w[i] = v[i];
  uint32_t kk = seed | 1;
  uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      if constexpr (KIND == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 3) asm volatile("v_min_u32 %0, %0, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 4) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 5) asm volatile("v_max_u32 %0, %0, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 6) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 7) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 8) asm volatile("v_and_b32 %0, %0, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 9) asm volatile("v_ashrrev_i32 %0, 31, %0" : "+v"(v[i]));
      if constexpr (KIND == 10) asm volatile("v_med3_u32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 11) asm volatile("v_sub_co_u32 %0, vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(kk) : "vcc");
      if constexpr (KIND == 12) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 13) asm volatile("v_sub_u32 %0, %0, %1 clamp" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 14) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 15) asm volatile("v_mov_b32 %0, %1" : "=v"(v[i]) : "v"(v[(i + 1) % CH]));
      if constexpr (KIND == 16) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 17) asm volatile("v_subrev_u32 %0, %1, %0" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 18) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(kk) : "vcc");
      if constexpr (KIND == 19) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(v[i]));
      if constexpr (KIND == 20) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(w[i]) : "v"(v[i]), "v"(kk) : "s0", "s1");
      if constexpr (KIND == 21) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(v[i]) : "v"(kk));
      if constexpr (KIND == 22) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(v[i]));
      if constexpr (KIND == 23) asm volatile("v_sub_co_u32 %0, s[2:3], %0, %1" : "+v"(v[i]) : "v"(kk) : "s2", "s3");
      if constexpr (KIND == 24) asm volatile("v_cndmask_b32 %0, %0, %1, s[4:5]" : "+v"(v[i]) : "v"(kk) : "s4", "s5");
      if constexpr (KIND == 25) asm volatile("v_mul_lo_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(kk));
    }
  }
  uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
  for (int i = 0; i < CH; i++) acc ^= v[i] ^ (uint32_t)w[i];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = c1 - c0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int KIND>
void run(const char *name, int ops_per_item, uint64_t *dclk, uint32_t *dout) {
  const int blocks = 2048;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  k<KIND><<<blocks, 256>>>(dclk, dout, 7);
  (void)hipEventRecord(e0);
  k<KIND><<<blocks, 256>>>(dclk, dout, 9);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  uint64_t *h = new uint64_t[2 * blocks];
  (void)hipMemcpy(h, dclk, 16 * blocks, hipMemcpyDeviceToHost);
  double c = 0, r = 0;
  for (int i = 0; i < blocks; i++) { c += h[2 * i]; r += h[2 * i + 1]; }
  double ghz = c / r * 0.1;  // memrealtime = 100 MHz
  double winstr = (double)blocks * 4 * ITERS * CH * ops_per_item;
  double cyc = ms * 1e-3 * ghz * 1e9 * 1024 / winstr;
  printf("%-26s %7.3f ms  clock %.2f GHz  %.2f cycles/wave-instr/SIMD  %.1f T lane-ops/s\n", name,
         ms, ghz, cyc, winstr * 64 / (ms * 1e-3) / 1e12);
  delete[] h;
}

int main() {
  uint64_t *dclk; uint32_t *dout;
  (void)hipMalloc(&dclk, 2048 * 16); (void)hipMalloc(&dout, 2048 * 256 * 4);
  run<15>("v_mov_b32", 1, dclk, dout);
  run<0>("v_add_u32", 1, dclk, dout);
  run<17>("v_subrev_u32", 1, dclk, dout);
  run<16>("v_xor_b32", 1, dclk, dout);
  run<8>("v_and_b32", 1, dclk, dout);
  run<19>("v_lshlrev_b32", 1, dclk, dout);
  run<9>("v_ashrrev_i32", 1, dclk, dout);
  run<3>("v_min_u32", 1, dclk, dout);
  run<5>("v_max_u32", 1, dclk, dout);
  run<10>("v_med3_u32", 1, dclk, dout);
  run<13>("v_sub_u32 clamp", 1, dclk, dout);
  run<6>("v_lshl_add_u32", 1, dclk, dout);
  run<7>("v_add3_u32", 1, dclk, dout);
  run<14>("v_pk_add_u16", 1, dclk, dout);
  run<12>("v_mul_u32_u24", 1, dclk, dout);
  run<1>("v_mul_lo_u32", 1, dclk, dout);
  run<2>("v_mul_hi_u32", 1, dclk, dout);
  run<4>("v_fma_f32", 1, dclk, dout);
  run<11>("v_sub_co+v_cndmask (pair)", 2, dclk, dout);
  run<18>("v_cmp+v_cndmask (pair)", 2, dclk, dout);
  run<20>("v_mad_u64_u32", 1, dclk, dout);
  run<21>("v_lshlrev_b32 (vgpr shift)", 1, dclk, dout);
  run<22>("v_lshrrev_b32", 1, dclk, dout);
  run<23>("v_sub_co_u32 (sgpr carry)", 1, dclk, dout);
  run<24>("v_cndmask_b32 (sgpr mask)", 1, dclk, dout);
  run<25>("v_mul_lo+v_add (pair)", 2, dclk, dout);
  return 0;
}
