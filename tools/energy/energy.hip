// Board energy of the work classes in the C3 product kernel (verdict r4 item 3: the C3 energy
// budget).  tools/energy/energy_microbench.py runs each kind back to back for a few seconds while it
// samples board power in process (amdsmi) and divides power by the kind's rate.
//   VALU kinds: CH independent chains per lane, 8 waves per SIMD, operands kept random by xor
//   feedback (round 4's chained v_mul_hi collapsed to zero, profiles/r4/energy/); a kind's
//   instruction energy = (ops per iteration x pair energy - the xor's) / its own count.
//   LDS kind: ds_write_b32 + ds_read_b32 of random words at lane-linear (conflict-free) addresses.
//   Memory kinds: four 16-byte non-temporal loads, stores or both per lane per iteration over
//   2 GiB buffers (HBM), or a 16-byte load from a 64 KiB table (the twiddles: L2 hits).
// Workgroups 0 .. blocks - 1 stamp s_memtime / s_memrealtime at entry and exit into a buffer of
// their own (in-kernel clock; nothing reads it on the device).
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC energy.hip -o libenergy.so
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CH 16
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

enum Kind {
  K_SLEEP, K_XOR, K_ADD, K_MULHI, K_MULLO, K_MAD64, K_CSUB, K_LDS, K_HBM_RD, K_HBM_WR, K_HBM_CP,
  K_L2_RD, K_COUNT
};

__device__ __forceinline__ void stamp(unsigned long long *t, unsigned long long *r) {
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(*t), "=s"(*r)::"memory");
}

template <int KIND>
__global__ __launch_bounds__(256) void ek(uint32_t *out, unsigned long long *stamps,
                                          const u4 *src, u4 *dst, size_t n16,
                                          uint32_t seed, int iters) {
  __shared__ uint32_t lds[CH * 256];
  uint32_t v[CH];
  uint64_t t[CH];
  uint32_t x = seed ^ (blockIdx.x * 0x9E3779B9u) ^ (threadIdx.x * 0x85EBCA6Bu);
#pragma unroll
  for (int i = 0; i < CH; i++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    v[i] = x;
    t[i] = ((uint64_t)x << 32) | (x * 0x2545F491u);
  }
  const uint32_t q = 2013265921u;
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) stamp(&t0, &r0);
  // (memory kinds: n16 and the grid are powers of two, so the sweep index is a mask)
  const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x, gsz = (size_t)gridDim.x * 256;
  const size_t mask = n16 - 1;
  u4 acc = {0, 0, 0, 0};
  for (int it = 0; it < iters; it++) {
    if constexpr (KIND == K_SLEEP) __builtin_amdgcn_s_sleep(2);
    if constexpr (KIND == K_XOR || KIND == K_ADD || KIND == K_MULHI || KIND == K_MULLO ||
                  KIND == K_MAD64 || KIND == K_CSUB) {
#pragma unroll
      for (int i = 0; i < CH; i++) {
        uint32_t &a = v[i];
        const uint32_t b = v[(i + 5) % CH];
        uint32_t tmp;
        if constexpr (KIND == K_XOR) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));
        if constexpr (KIND == K_ADD) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
        if constexpr (KIND == K_MULHI)
          asm volatile("v_mul_hi_u32 %1, %0, %2\n\tv_xor_b32 %0, %0, %1" : "+v"(a), "=&v"(tmp) : "v"(b));
        if constexpr (KIND == K_MULLO)
          asm volatile("v_mul_lo_u32 %1, %0, %2\n\tv_xor_b32 %0, %0, %1" : "+v"(a), "=&v"(tmp) : "v"(b));
        if constexpr (KIND == K_MAD64) {  // carry-out to a dead SGPR pair, as the compiler's own
          asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(t[i]) : "v"(a), "v"(b) : "s0", "s1");
          asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"((uint32_t)(t[i] >> 32)));
        }
        if constexpr (KIND == K_CSUB)   // x - q with borrow, select, then xor-refresh of x
          asm volatile("v_sub_co_u32 %1, s[0:1], %0, %2\n\ts_nop 1\n\t"
                       "v_cndmask_b32_e64 %1, %1, %0, s[0:1]\n\tv_xor_b32 %0, %1, %3"
                       : "+v"(a), "=&v"(tmp) : "v"(q), "v"(b) : "s0", "s1");
      }
    }
    if constexpr (KIND == K_LDS) {
#pragma unroll
      for (int i = 0; i < CH; i++) {
        lds[i * 256 + threadIdx.x] = v[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t r = lds[i * 256 + (threadIdx.x ^ 1)];
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[i]) : "v"(r));
      }
    }
    if constexpr (KIND == K_HBM_RD || KIND == K_HBM_CP || KIND == K_HBM_WR) {
      // four 16-byte accesses per lane per iteration (in flight together), sweeping 2 GiB
      u4 w[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const size_t i = (gid + ((size_t)it * 4 + u) * gsz) & mask;
        if constexpr (KIND == K_HBM_WR) w[u] = u4{v[u] + it, v[u + 4], v[u + 8] ^ it, v[u + 12]};
        else w[u] = __builtin_nontemporal_load(src + i);
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const size_t i = (gid + ((size_t)it * 4 + u) * gsz) & mask;
        if constexpr (KIND == K_HBM_RD) acc ^= w[u];
        else __builtin_nontemporal_store(w[u], dst + i);
      }
    }
    if constexpr (KIND == K_L2_RD) {  // 64 KiB table: 4096 uint4, L2-resident like the twiddles
      const u4 w = src[(gid * 7 + (size_t)it * 131) & 4095];
      acc.x ^= w.x; acc.y ^= w.y; acc.z ^= w.z; acc.w ^= w.w;
    }
  }
  if (threadIdx.x == 0) {
    unsigned long long t1, r1;
    stamp(&t1, &r1);
    stamps[blockIdx.x * 4 + 0] = t0; stamps[blockIdx.x * 4 + 1] = r0;
    stamps[blockIdx.x * 4 + 2] = t1; stamps[blockIdx.x * 4 + 3] = r1;
  }
  uint32_t s = acc.x ^ acc.y ^ acc.z ^ acc.w;
#pragma unroll
  for (int i = 0; i < CH; i++) s ^= v[i] ^ (uint32_t)t[i] ^ (uint32_t)(t[i] >> 32);
  out[gid] = s;
}

extern "C" {
int en_kinds() { return K_COUNT; }
const char *en_name(int k) {
  static const char *n[] = {"sleep", "v_xor_b32", "v_add_u32", "v_mul_hi_u32+xor", "v_mul_lo_u32+xor",
                            "v_mad_u64_u32+xor", "v_sub_co+v_cndmask+xor", "ds_write_b32+ds_read_b32+xor",
                            "hbm_read_16B_nt", "hbm_write_16B_nt", "hbm_copy_16B_nt", "l2_read_16B"};
  return k >= 0 && k < K_COUNT ? n[k] : "";
}
// VALU instructions per lane per iteration (including the xor refresh), LDS instructions, bytes
// moved to / from HBM (or L2) per lane per iteration
int en_valu_per_iter(int k) {
  switch (k) {
    case K_XOR: case K_ADD: return CH;
    case K_MULHI: case K_MULLO: case K_MAD64: return 2 * CH;
    case K_CSUB: return 3 * CH;
    case K_LDS: return CH;
    default: return 0;
  }
}
int en_lds_per_iter(int k) { return k == K_LDS ? 2 * CH : 0; }
int en_bytes_per_iter(int k) {
  return k == K_HBM_RD || k == K_HBM_WR ? 64 : k == K_HBM_CP ? 128 : k == K_L2_RD ? 16 : 0;
}
int en_launch(int kind, void *out, void *stamps, const void *src, void *dst, size_t n16, int blocks,
              int iters, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  uint32_t *o = (uint32_t *)out;
  unsigned long long *st = (unsigned long long *)stamps;
#define L(K) case K: hipLaunchKernelGGL(ek<K>, dim3(blocks), dim3(256), 0, s, o, st, (const u4 *)src, (u4 *)dst, n16, 12345u + K, iters); break
  switch (kind) {
    L(0); L(1); L(2); L(3); L(4); L(5); L(6); L(7); L(8); L(9); L(10); L(11);
    default: return -1;
  }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
}
