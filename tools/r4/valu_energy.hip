// Energy per VALU instruction on gfx950 at the package power cap (verdict r3 item 3: the FP64-FMA
// and 24-bit-multiply levers for the butterfly's modular products, never priced in energy).
// Each kind issues one instruction type in CH independent chains per lane, 8 waves per SIMD, on
// random operands; tools/r4/valu_energy.py runs every kind back to back for a few seconds while
// it samples board power, and divides power by the lane-op rate.  Block 0..blocks-1 also stamp
// s_memtime / s_memrealtime around their loop (a buffer of their own; no output depends on
// them), so the clock each kind runs at is read in-kernel.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC valu_energy.hip -o libvalu_energy.so
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CH 16

__device__ __forceinline__ unsigned long long stamp_t() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
__device__ __forceinline__ unsigned long long stamp_r() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

#define OP1(ins) asm volatile(ins " %0, %0, %1" : "+v"(v[i]) : "v"(k))
template <int KIND>
__global__ __launch_bounds__(256) void ve(uint32_t *out, unsigned long long *stamps,
                                          uint32_t seed, int iters) {
  uint32_t v[CH];
  uint64_t t[CH];
  double d[CH];
  float f[CH];
  uint32_t x = seed ^ (blockIdx.x * 0x9E3779B9u) ^ (threadIdx.x * 0x85EBCA6Bu);
#pragma unroll
  for (int i = 0; i < CH; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    v[i] = x;
    t[i] = ((uint64_t)x << 32) | (x * 0x2545F491u);
    d[i] = 1.0 + (double)(x & 0xFFFFF) * 0x1p-21;
    f[i] = 1.0f + (float)(x & 0xFFFF) * 0x1p-17f;
  }
  x ^= x << 13; x ^= x >> 17; x ^= x << 5;
  const uint32_t k = x | 1u;
  const double dk = 1.0 + (double)(k & 0xFFF) * 0x1p-40;
  const float fk = 1.0f + (float)(k & 0xFF) * 0x1p-30f;
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = stamp_t(); r0 = stamp_r(); }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      if constexpr (KIND == 0) OP1("v_add_u32");
      if constexpr (KIND == 1) OP1("v_mul_lo_u32");
      if constexpr (KIND == 2) OP1("v_mul_hi_u32");
      if constexpr (KIND == 3)  // 64-bit multiply-add chain, carry-out to a dead SGPR pair
        asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(t[i]) : "v"(v[i]), "v"(k) : "s0", "s1");
      if constexpr (KIND == 4) OP1("v_mul_u32_u24");
      if constexpr (KIND == 5)
        asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(v[i]) : "v"(v[(i + 1) % CH]), "v"(k));
      if constexpr (KIND == 6) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(dk));
      if constexpr (KIND == 7) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(dk));
      if constexpr (KIND == 8) {  // conditional subtraction: v_sub_co (VOP3, carry to SGPRs) + select
        uint32_t dd;
        asm volatile("v_sub_co_u32 %0, s[0:1], %1, %2\n\ts_nop 1\n\tv_cndmask_b32_e64 %1, %0, %1, s[0:1]"
                     : "=&v"(dd), "+v"(v[i]) : "v"(k) : "s0", "s1");
      }
      if constexpr (KIND == 9) OP1("v_xor_b32");
      if constexpr (KIND == 10) { if (i == 0) __builtin_amdgcn_s_sleep(2); }
      if constexpr (KIND == 11) OP1("v_mul_hi_u32_u24");
      if constexpr (KIND == 12) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[i]) : "v"(fk));
      if constexpr (KIND == 13) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(v[i]) : "v"(k));
      // (kinds 2 and 11 chain v = mulhi(v, k), which shrinks v towards 0 within a few steps, so
      // their operands stop toggling and their energy reads low; kinds 14-16 keep the operands
      // random with v ^= op(v, k): energy(op) = 2 x pair - energy(v_xor_b32))
      if constexpr (KIND == 14 || KIND == 15 || KIND == 16) {
        uint32_t tmp;
        if constexpr (KIND == 14)
          asm volatile("v_mul_hi_u32 %1, %0, %2\n\tv_xor_b32 %0, %0, %1" : "+v"(v[i]), "=&v"(tmp) : "v"(k));
        if constexpr (KIND == 15)
          asm volatile("v_mul_hi_u32_u24 %1, %0, %2\n\tv_xor_b32 %0, %0, %1" : "+v"(v[i]), "=&v"(tmp) : "v"(k));
        if constexpr (KIND == 16)
          asm volatile("v_mul_lo_u32 %1, %0, %2\n\tv_xor_b32 %0, %0, %1" : "+v"(v[i]), "=&v"(tmp) : "v"(k));
      }
    }
  }
  if (threadIdx.x == 0) {
    const unsigned long long t1 = stamp_t(), r1 = stamp_r();
    stamps[blockIdx.x * 4 + 0] = t0; stamps[blockIdx.x * 4 + 1] = r0;
    stamps[blockIdx.x * 4 + 2] = t1; stamps[blockIdx.x * 4 + 3] = r1;
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < CH; i++)
    acc ^= v[i] ^ (uint32_t)t[i] ^ (uint32_t)(t[i] >> 32) ^ (uint32_t)(int64_t)d[i] ^ (uint32_t)f[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

extern "C" {
int ve_kinds() { return 17; }
const char *ve_name(int kind) {
  static const char *n[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32",
                            "v_mul_u32_u24", "v_mad_u32_u24", "v_fma_f64", "v_mul_f64",
                            "v_sub_co_u32+v_cndmask_b32 (pair)", "v_xor_b32", "s_sleep (no VALU)",
                            "v_mul_hi_u32_u24", "v_fma_f32", "v_lshl_add_u32",
                            "v_mul_hi_u32+v_xor_b32 (pair, random operands)",
                            "v_mul_hi_u32_u24+v_xor_b32 (pair, random operands)",
                            "v_mul_lo_u32+v_xor_b32 (pair, random operands)"};
  return kind >= 0 && kind < 17 ? n[kind] : "";
}
// VALU instructions per lane per loop iteration
int ve_ops_per_iter(int kind) { return kind == 8 || kind >= 14 ? 2 * CH : kind == 10 ? 0 : CH; }
int ve_launch(int kind, void *out, void *stamps, int blocks, int iters, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  uint32_t *o = (uint32_t *)out;
  unsigned long long *st = (unsigned long long *)stamps;
#define L(K) case K: hipLaunchKernelGGL(ve<K>, dim3(blocks), dim3(256), 0, s, o, st, 12345u + K, iters); break
  switch (kind) {
    L(0); L(1); L(2); L(3); L(4); L(5); L(6); L(7); L(8); L(9); L(10); L(11); L(12); L(13);
    L(14); L(15); L(16);
    default: return -1;
  }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
}
