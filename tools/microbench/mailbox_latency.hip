// mailbox_latency -- transport cost of one small host transaction (the device server's protocol,
// nttmul.cpp run_server) with the request mailbox in two places:
//   H: go, a, b in pinned host memory; the resident wave polls go and pulls a, b across PCIe
//      (every poll and every operand load a PCIe read round trip) -- the round-4 server;
//   V: go, a, b in device memory the host can map (large BAR); the host pushes them with posted
//      writes and the wave polls and loads its own HBM.
// c goes back to pinned host memory in both (posted writes; the host spins on c itself: a word
// that no longer holds the pending marker has landed).  The kernel's "product" is c = a ^ b, so
// what is timed is the transport.  Also reports which allocation gives a host-writable device
// pointer.  Every spin is bounded: the wave leaves on stop, after 1 s, or after 20 ms idle.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

constexpr int kWords = 512;  // a, b, c: n = 256 x 2 products, or n = 512
constexpr unsigned kPending = 0xFFFFFFFFu;
struct Req {
  alignas(128) unsigned go;
  alignas(128) unsigned a[kWords];
  alignas(128) unsigned b[kWords];
};
struct Resp {
  alignas(128) unsigned c[kWords];
};

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, (int)bytes, 0x00020000);
}

// one wave: poll go, load a and b (words per request), c = a ^ b to host memory
template <int MODE, bool FENCE = true>
__global__ __launch_bounds__(64) void k_serve(Req *rq, Resp *rs, int words, unsigned spin,
                                              unsigned long long idle, unsigned long long life) {
  __shared__ uint4 sa[kWords / 4], sb[kWords / 4];
  const int lane = threadIdx.x;
  unsigned seen = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long last = t0;
  const auto ra = rsrc(rq->a, kWords * 4), rb = rsrc(rq->b, kWords * 4), rc = rsrc(rs->c, kWords * 4);
  for (;;) {
    unsigned go = seen;
    const auto poll = [&]() {
      const unsigned v = __hip_atomic_load(&rq->go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_sched_barrier(0);
      return v;
    };
    const auto gone = [&]() {
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      return now - last > idle || now - t0 > life;
    };
    if constexpr (MODE >= 1) {  // several polls in flight: 3, s_sleep 16 apart (MODE 1) or 4, s_sleep 1 apart (MODE 2)
      constexpr int SL = MODE == 1 ? 16 : 1;
      unsigned p0 = poll();
      __builtin_amdgcn_s_sleep(SL);
      unsigned p1 = poll();
      __builtin_amdgcn_s_sleep(SL);
      unsigned p2 = MODE == 2 ? poll() : 0u;
      if (MODE == 2) __builtin_amdgcn_s_sleep(SL);
      bool quit = false;
      for (;;) {
        unsigned p3 = poll();
        if ((go = __builtin_amdgcn_readfirstlane(p0)) != seen) break;
        if ((quit = gone())) break;
        __builtin_amdgcn_s_sleep(SL);
        p0 = poll();
        if ((go = __builtin_amdgcn_readfirstlane(p1)) != seen) break;
        if ((quit = gone())) break;
        __builtin_amdgcn_s_sleep(SL);
        p1 = poll();
        if (MODE == 2) {
          if ((go = __builtin_amdgcn_readfirstlane(p2)) != seen) break;
          if ((quit = gone())) break;
          __builtin_amdgcn_s_sleep(SL);
          p2 = poll();
        }
        if ((go = __builtin_amdgcn_readfirstlane(p3)) != seen) break;
        if ((quit = gone())) break;
        __builtin_amdgcn_s_sleep(SL);
      }
      if (quit) return;
    } else {
      for (;;) {
        go = __builtin_amdgcn_readfirstlane(poll());
        if (go != seen) break;
        if (gone()) return;
        __builtin_amdgcn_s_sleep(2);
      }
    }
    if (go == 0xFFFFFFFFu) return;  // stop
    if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // (the loads below are sc0 sc1)
    const int q4 = words / 4;
    for (int i = lane; i < q4; i += 64) {  // system-scope (sc0 sc1) 16-byte loads
      auto va = __builtin_amdgcn_raw_buffer_load_b128(ra, i * 16, 0, 17);
      auto vb = __builtin_amdgcn_raw_buffer_load_b128(rb, i * 16, 0, 17);
      sa[i] = make_uint4(va[0], va[1], va[2], va[3]);
      sb[i] = make_uint4(vb[0], vb[1], vb[2], vb[3]);
    }
    __syncthreads();
    if (spin) {  // stand-in for the product's compute time
      const unsigned long long s0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - s0 < spin) __builtin_amdgcn_s_sleep(1);
    }
    for (int i = lane; i < q4; i += 64) {
      const uint4 x = sa[i], y = sb[i];
      __attribute__((ext_vector_type(4))) unsigned w = {x.x ^ y.x, x.y ^ y.y, x.z ^ y.z, x.w ^ y.w};
      __builtin_amdgcn_raw_buffer_store_b128(w, rc, i * 16, 0, 17);  // write-through
    }
    __syncthreads();
    seen = go;
    last = __builtin_amdgcn_s_memrealtime();
  }
}

// a chain of n dependent system-scope loads of go (the next address depends on the last value)
__global__ void k_chain(Req *rq, unsigned long long *out, int n) {
  unsigned v = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; i++)
    v = __hip_atomic_load(&rq->go + (v & 0x80000000u ? 1 : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) *out = (t1 - t0) + (v == 0x12345678u);
}

static double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(p * (v.size() - 1))];
}

// host side of one variant: rq is what the host writes through (host or mapped device pointer),
// drq what the kernel sees
static void run(const char *name, Req *rq, Req *drq, Resp *rs, Resp *drs, int words, int calls,
                bool wc_fence, int stagger = 0, unsigned spin = 0, bool fence = true) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  rq->go = 0;
  _mm_sfence();
  if (!fence)
    hipLaunchKernelGGL((k_serve<0, false>), dim3(1), dim3(64), 0, s, drq, drs, words, spin, 2000000ull, 100000000ull);
  else if (stagger == 2)
    hipLaunchKernelGGL(k_serve<2>, dim3(1), dim3(64), 0, s, drq, drs, words, spin, 2000000ull, 100000000ull);
  else if (stagger == 1)
    hipLaunchKernelGGL(k_serve<1>, dim3(1), dim3(64), 0, s, drq, drs, words, spin, 2000000ull, 100000000ull);
  else
    hipLaunchKernelGGL(k_serve<0>, dim3(1), dim3(64), 0, s, drq, drs, words, spin, 2000000ull, 100000000ull);
  std::vector<unsigned> a(kWords), b(kWords);
  std::vector<double> us, us_w;
  unsigned seq = 0;
  int bad = 0, lost = 0;
  for (int it = 0; it < calls + 50; it++) {
    for (int i = 0; i < words; i++) a[i] = it * 7919u + i, b[i] = i * 31u;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < words; i++) rs->c[i] = kPending;
    memcpy(rq->a, a.data(), words * 4);
    memcpy(rq->b, b.data(), words * 4);
    if (wc_fence) _mm_sfence();  // WC / UC mapping: the data ahead of go
    __atomic_store_n(&rq->go, ++seq, __ATOMIC_RELEASE);
    if (wc_fence) _mm_sfence();
    const auto tw = std::chrono::steady_clock::now();
    const auto t_lim = t0 + std::chrono::seconds(2);
    for (;;) {
      bool all = true;
      for (int i = 0; i < words && all; i++)
        all = __atomic_load_n(&rs->c[i], __ATOMIC_RELAXED) != kPending;
      if (all) break;
      _mm_pause();
      if (std::chrono::steady_clock::now() > t_lim) { lost = 1; break; }
    }
    if (lost) break;
    const auto t1 = std::chrono::steady_clock::now();
    for (int i = 0; i < words; i++) bad += rs->c[i] != (a[i] ^ b[i]);
    if (it >= 50) {
      us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      us_w.push_back(std::chrono::duration<double, std::micro>(tw - t0).count());
    }
  }
  rq->go = 0xFFFFFFFFu;
  _mm_sfence();
  CK(hipStreamSynchronize(s));
  CK(hipStreamDestroy(s));
  if (lost) {
    printf("{\"variant\": \"%s\", \"words\": %d, \"error\": \"no answer within 2 s\"}\n", name, words);
    return;
  }
  printf("{\"variant\": \"%s\", \"poll\": \"%s\", \"spin_us\": %.2f, \"words\": %d, \"calls\": %d, "
         "\"bad_words\": %d, \"us_p10\": %.2f, \"us_p50\": %.2f, \"us_p90\": %.2f, \"host_write_us_p50\": %.2f}\n",
         name, !fence ? "1, s_sleep 2, no acquire fence" : stagger == 2 ? "4 in flight, s_sleep 1" : stagger ? "3 in flight, s_sleep 16" : "1, s_sleep 2", spin / 100.0, words, calls, bad,
         pct(us, 0.1), pct(us, 0.5), pct(us, 0.9), pct(us_w, 0.5));
}

static hsa_agent_t g_cpu, g_gpu;
static int g_ngpu;
static hsa_status_t agent_cb(hsa_agent_t a, void *) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
  if (t == HSA_DEVICE_TYPE_GPU && g_ngpu++ == 0) g_gpu = a;
  return HSA_STATUS_SUCCESS;
}
static hsa_amd_memory_pool_t g_pool;
static hsa_status_t pool_cb(hsa_amd_memory_pool_t p, void *want) {
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t fl = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
  if ((fl & *(uint32_t *)want) && !g_pool.handle) g_pool = p;
  return HSA_STATUS_SUCCESS;
}

static void *host_view(void *dptr) {
  hsa_amd_pointer_info_t info;
  memset(&info, 0, sizeof(info));
  info.size = sizeof(info);
  if (hsa_amd_pointer_info(dptr, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return nullptr;
  return info.hostBaseAddress;
}

int main(int argc, char **argv) {
  const int calls = argc > 1 ? atoi(argv[1]) : 2000;
  hsa_init();
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  Resp *rs;
  CK(hipHostMalloc((void **)&rs, sizeof(Resp), hipHostMallocCoherent));
  Resp *drs;
  CK(hipHostGetDevicePointer((void **)&drs, rs, 0));

  // H: the round-4 mailbox
  Req *hq, *dhq;
  CK(hipHostMalloc((void **)&hq, sizeof(Req), hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void **)&dhq, hq, 0));
  memset(hq, 0, sizeof(Req));
  for (int w : {256, 512}) run("host_mailbox", hq, dhq, rs, drs, w, calls, false);
  for (int rep = 0; rep < 2; rep++) {
    run("host_mailbox", hq, dhq, rs, drs, 256, calls, false, 0, 0, true);
    run("host_mailbox", hq, dhq, rs, drs, 256, calls, false, 0, 0, false);
  }

  // V1: fine-grained device memory from HIP; the host's view from the pointer attributes / HSA
  Req *fq = nullptr;
  hipError_t e = hipExtMallocWithFlags((void **)&fq, sizeof(Req), hipDeviceMallocFinegrained);
  void *hv = nullptr;
  if (e == hipSuccess) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, fq) == hipSuccess) hv = at.hostPointer;
    void *hv2 = host_view(fq);
    printf("{\"alloc\": \"hipExtMallocWithFlags(Finegrained)\", \"dptr\": \"%p\", \"hip_host_ptr\": \"%p\", "
           "\"hsa_host_base\": \"%p\"}\n", (void *)fq, hv, hv2);
    if (!hv) hv = hv2;
  } else {
    printf("{\"alloc\": \"hipExtMallocWithFlags(Finegrained)\", \"error\": \"%s\"}\n", hipGetErrorString(e));
  }
  // V2: HSA fine-grained VRAM pool, CPU agent granted access
  hsa_iterate_agents(agent_cb, nullptr);
  uint32_t want = HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED;
  hsa_amd_agent_iterate_memory_pools(g_gpu, pool_cb, &want);
  void *sq = nullptr, *shv = nullptr;
  if (g_pool.handle) {
    hsa_status_t hs = hsa_amd_memory_pool_allocate(g_pool, sizeof(Req), 0, &sq);
    hsa_status_t ha = HSA_STATUS_ERROR;
    if (hs == HSA_STATUS_SUCCESS) {
      hsa_agent_t ags[2] = {g_gpu, g_cpu};
      ha = hsa_amd_agents_allow_access(2, ags, nullptr, sq);
      shv = host_view(sq);
    }
    printf("{\"alloc\": \"hsa fine-grained VRAM pool + CPU access\", \"alloc_status\": %d, \"allow_status\": %d, "
           "\"dptr\": \"%p\", \"hsa_host_base\": \"%p\"}\n", (int)hs, (int)ha, sq, shv);
  }
  fflush(stdout);
  // the host writes through its view; a probe write/read first (a fault here is the host's own)
  struct V { const char *name; Req *host; Req *dev; } vs[2] = {{"vram_hip_finegrained", (Req *)hv, fq},
                                                              {"vram_hsa_pool", (Req *)shv, (Req *)sq}};
  for (auto &v : vs) {
    if (!v.host || !v.dev) continue;
    v.host->go = 0;
    v.host->a[0] = 12345;
    _mm_sfence();
    unsigned back = 0;
    CK(hipMemcpy(&back, &v.dev->a[0], 4, hipMemcpyDeviceToHost));
    printf("{\"variant\": \"%s\", \"probe_readback\": %u}\n", v.name, back);
    fflush(stdout);
    if (back != 12345) continue;
    for (int w : {256, 512}) run(v.name, v.host, v.dev, rs, drs, w, calls, true);
    if (v.dev != fq) continue;
    for (int rep = 0; rep < 3; rep++) {
      run(v.name, v.host, v.dev, rs, drs, 256, calls, true, 0, 0, true);
      run(v.name, v.host, v.dev, rs, drs, 256, calls, true, 0, 0, false);
    }
    for (int st : {2, 1}) run(v.name, v.host, v.dev, rs, drs, 256, calls, true, st, 0);
    // latency of one system-scope load of the device-memory go word: a dependent chain
    {
      unsigned long long *d_t;
      CK(hipMalloc(&d_t, 8));
      hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, v.dev, d_t, 256);
      unsigned long long tk = 0;
      CK(hipMemcpy(&tk, d_t, 8, hipMemcpyDeviceToHost));
      printf("{\"variant\": \"%s\", \"poll_load_latency_ns\": %.1f}\n", v.name, tk * 10.0 / 256);
      CK(hipFree(d_t));
    }
  }
  return 0;
}
