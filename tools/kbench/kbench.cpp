// kbench — standalone timing driver for the polymul kernels (no Python, no torch), used for
// ablation builds (-DNTTMUL_ABL_*) and quick A/B runs on the GPU box.
//   kbench <n> <q> <batch> [reps] [io_bits]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "kb.hpp"
#include "launch.hpp"
#include "planner.hpp"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

int main(int argc, char **argv) {
  uint32_t n = argc > 1 ? atoi(argv[1]) : 4096;
  uint64_t q = argc > 2 ? strtoull(argv[2], 0, 0) : 2013265921ull;
  size_t batch = argc > 3 ? strtoull(argv[3], 0, 0) : 65536;
  int reps = argc > 4 ? atoi(argv[4]) : 20;
  nttmul::Plan P;
  if (nttmul::make_plan(n, q, 0, &P)) { fprintf(stderr, "bad plan\n"); return 1; }
  int io_bits = argc > 5 ? atoi(argv[5]) : (q < (1ull << 32) ? 32 : 64);
  size_t wb = io_bits / 8, bytes = batch * n * wb;
  void *a, *b, *c, *fw, *iw, *scr[4] = {0, 0, 0, 0};
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes)); CK(hipMalloc(&c, bytes));
  CK(hipMalloc(&fw, P.fw.size())); CK(hipMalloc(&iw, P.iw.size()));
  CK(hipMemcpy(fw, P.fw.data(), P.fw.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(iw, P.iw.data(), P.iw.size(), hipMemcpyHostToDevice));
  if (P.logn > 12) {
    for (int i = 0; i < 3; i++) CK(hipMalloc(&scr[i], batch * n * (P.word_bits / 8)));
    CK(hipMalloc(&scr[3], kb::mp_sync_bytes(batch)));
  }
  nttmul::LaunchTables T;
  T.logn = P.logn; T.word_bits = P.word_bits; T.q = P.q; T.qinv_neg = P.qinv_neg;
  T.f = P.f; T.fs = P.fs; T.wf = P.wf; T.wfs = P.wfs; T.fw = fw; T.iw = iw;
  T.f4 = P.f4; T.f4s = P.f4s; T.wf4 = P.wf4; T.wf4s = P.wf4s;
  T.f8 = P.f8; T.f8s = P.f8s; T.wf8 = P.wf8; T.wf8s = P.wf8s;
  T.fi = P.fi; T.fis = P.fis; T.wfi = P.wfi; T.wfis = P.wfis; T.r2 = P.r2;
  CK(hipDeviceGetAttribute(&T.cus, hipDeviceAttributeMultiprocessorCount, 0));
  // KB_PRIO: the issue-priority variant as nttmul_params.issue_prio (-1 never, 0 automatic, 1 always)
  T.prio = getenv("KB_PRIO") ? atoi(getenv("KB_PRIO")) : 0;
  kb::Conf C;
  // KB_MP_LAG > 0: n > 4096 products as one persistent launch (k_mp_persist) with this lag
  C.mp_lag = getenv("KB_MP_LAG") ? atoi(getenv("KB_MP_LAG")) : 0;
  // KB_PIPE: n = 1024 products through k_rows_pipe with KB_PIPE products per wave (> 0),
  // k_rows_w4 (-1) or k_rows_ab (-2)
  C.pipe_per_wave = getenv("KB_PIPE") ? atoi(getenv("KB_PIPE")) : 0;
  if (C.mp_lag > 0 && P.logn > 12) CK(hipMemset(scr[3], 0, kb::mp_sync_bytes(batch)));
  unsigned long long *stats = nullptr;
#if NTTMUL_MP_STATS
  CK(hipMalloc(&stats, 9 * 8));
  CK(hipMemset(stats, 0, 9 * 8));
  C.mp_stats = stats;
#endif
  CK(kb::fill(a, b, P.logn, q, 0x4E54544D554Cull, batch, io_bits, 0));
  // KB_ROTATE=R: the timed launches cycle over R (a, b, c) sets with identical inputs, so a batch
  // smaller than the 256 MiB Infinity Cache is read from HBM (as bench.py --rotate)
  const int rot = getenv("KB_ROTATE") ? atoi(getenv("KB_ROTATE")) : 1;
  void *ra[64], *rb[64], *rc[64];
  ra[0] = a; rb[0] = b; rc[0] = c;
  for (int i = 1; i < rot && i < 64; i++) {
    CK(hipMalloc(&ra[i], bytes)); CK(hipMalloc(&rb[i], bytes)); CK(hipMalloc(&rc[i], bytes));
    CK(kb::fill(ra[i], rb[i], P.logn, q, 0x4E54544D554Cull, batch, io_bits, 0));
  }
  // KB_ROWS_LDS=B: the row pass of an n > 4096 product takes B more bytes of LDS per workgroup
  // (caps its workgroups per CU, so column-pass waves can be resident beside it)
  C.rows_lds_extra = getenv("KB_ROWS_LDS") ? atoi(getenv("KB_ROWS_LDS")) : 0;
  // KB_SUB=S (n > 4096): the batch runs as sub-batches of S products through a ring of three
  // scratch sets, the row passes on one stream and the column passes on another, issued so that
  // the columns of sub-batch i + 1 and the inverse columns of i - 1 can overlap the rows of i
  const size_t sub = getenv("KB_SUB") ? strtoull(getenv("KB_SUB"), 0, 0) : 0;
  if (sub) {
    if (P.logn <= 12 || batch % sub) { fprintf(stderr, "KB_SUB needs n > 4096 and sub | batch\n"); return 1; }
    for (int i = 0; i < 3; i++) CK(hipFree(scr[i]));
  }
  void *ring[3][3];
  hipStream_t scol = 0, srow = 0;
  constexpr int kEv = 16;
  hipEvent_t evcf[kEv], evr[kEv];
  size_t gsub = 0;  // sub-batches issued so far (ring position)
  if (sub) {
    for (int r = 0; r < 3; r++)
      for (int i = 0; i < 3; i++) CK(hipMalloc(&ring[r][i], sub * n * (P.word_bits / 8)));
    // KB_COL_CUS=k: spatial partition instead of co-residency -- the column stream may use CUs
    // [0, k), the row stream the others (hipExtStreamCreateWithCUMask; 0 = both use every CU)
    const int col_cus = getenv("KB_COL_CUS") ? atoi(getenv("KB_COL_CUS")) : 0;
    if (col_cus > 0) {
      int ncu = 0;
      CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
      std::vector<uint32_t> mc((ncu + 31) / 32, 0), mr((ncu + 31) / 32, 0);
      for (int cu = 0; cu < ncu; cu++) (cu < col_cus ? mc : mr)[cu / 32] |= 1u << (cu % 32);
      CK(hipExtStreamCreateWithCUMask(&scol, (uint32_t)mc.size(), mc.data()));
      CK(hipExtStreamCreateWithCUMask(&srow, (uint32_t)mr.size(), mr.data()));
      printf("  column stream on CUs [0, %d), row stream on [%d, %d)\n", col_cus, col_cus, ncu);
    } else {
      CK(hipStreamCreateWithFlags(&scol, hipStreamNonBlocking));
      CK(hipStreamCreateWithFlags(&srow, hipStreamNonBlocking));
    }
    for (int i = 0; i < kEv; i++) {
      CK(hipEventCreateWithFlags(&evcf[i], hipEventDisableTiming));
      CK(hipEventCreateWithFlags(&evr[i], hipEventDisableTiming));
    }
  }
  auto pipelined = [&](void *pa, void *pb, void *pc) {
    const size_t ns = batch / sub, step = sub * n * wb;
    auto pass = [&](int phase, size_t g, size_t i, hipStream_t s) {
      kb::Conf c = C;
      c.mp_phase = phase;
      void *r4[4] = {ring[g % 3][0], ring[g % 3][1], ring[g % 3][2], nullptr};
      CK(kb::launch(T, c, (char *)pa + i * step, (char *)pb + i * step, (char *)pc + i * step,
                    sub, io_bits, r4, s));
    };
    pass(0, gsub, 0, scol);
    CK(hipEventRecord(evcf[gsub % kEv], scol));
    for (size_t i = 0; i < ns; i++) {
      const size_t g = gsub + i;
      CK(hipStreamWaitEvent(srow, evcf[g % kEv], 0));
      pass(1, g, i, srow);
      CK(hipEventRecord(evr[g % kEv], srow));
      if (i + 1 < ns) {
        pass(0, g + 1, i + 1, scol);
        CK(hipEventRecord(evcf[(g + 1) % kEv], scol));
      }
      CK(hipStreamWaitEvent(scol, evr[g % kEv], 0));
      pass(2, g, i, scol);
    }
    gsub += ns;
  };
  if (sub) {
    CK(hipDeviceSynchronize());  // the fills ran on the null stream
    for (int i = 0; i < 3; i++) pipelined(a, b, c);
    CK(hipDeviceSynchronize());
  } else {
    for (int i = 0; i < 3; i++) CK(kb::launch(T, C, a, b, c, batch, io_bits, scr, 0));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  // KB_STREAMS=2: consecutive launches alternate over two streams with their own c buffer (a and
  // b are read-only), so one launch's tail overlaps the next one's ramp
  const int nstreams = getenv("KB_STREAMS") ? atoi(getenv("KB_STREAMS")) : 1;
  hipStream_t st[2] = {0, 0};
  void *c2 = c;
  hipEvent_t join;
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  if (nstreams == 2) {
    CK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking));
    CK(hipMalloc(&c2, bytes));
    CK(hipDeviceSynchronize());
  }
  if (!sub) CK(hipEventRecord(e0, st[0]));
  if (nstreams == 2) {
    CK(hipEventRecord(join, st[0]));
    CK(hipStreamWaitEvent(st[1], join, 0));
  }
  if (sub) {  // the column stream times the run; the row stream joins it at both ends
    CK(hipEventRecord(e0, scol));
    CK(hipStreamWaitEvent(srow, e0, 0));
    for (int i = 0; i < reps; i++) pipelined(a, b, c);
    CK(hipEventRecord(join, srow));
    CK(hipStreamWaitEvent(scol, join, 0));
    st[0] = scol;
    reps = -reps;  // (skip the loop below)
  }
  for (int i = 0; i < reps; i++) {
    const int k = nstreams == 2 ? (i & 1) : 0;
    if (rot > 1) {
      const int r = i % (rot < 64 ? rot : 64);
      CK(kb::launch(T, C, ra[r], rb[r], rc[r], batch, io_bits, scr, st[k]));
      continue;
    }
    CK(kb::launch(T, C, a, b, k ? c2 : c, batch, io_bits, scr, st[k]));
  }
  if (nstreams == 2) {
    CK(hipEventRecord(join, st[1]));
    CK(hipStreamWaitEvent(st[0], join, 0));
  }
  CK(hipEventRecord(e1, st[0]));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  if (reps < 0) reps = -reps;
  ms /= reps;
  double pps = batch / (ms * 1e-3);
  double gbs = 3.0 * n * wb * batch / (ms * 1e-3) / 1e9;
  // checksum of c so variants can be compared for identical output
  unsigned long long sum = 0;
  {
    size_t cnt = bytes / 8;
    unsigned long long *h = (unsigned long long *)malloc(bytes);
    CK(hipMemcpy(h, c, bytes, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < cnt; i++) sum = sum * 1099511628211ull + h[i];
    free(h);
  }
  unsigned fault = 0;
  if (C.mp_lag > 0 && P.logn > 12) CK(hipMemcpy(&fault, (unsigned *)scr[3] + 1, 4, hipMemcpyDeviceToHost));
  if (fault) printf("FAULT: k_mp_persist poll gave up\n");
  if (stats) {
    unsigned long long h[9];
    CK(hipMemcpy(h, stats, sizeof(h), hipMemcpyDeviceToHost));
    const char *nm[3] = {"CI", "R", "CF"};
    for (int k = 0; k < 3; k++)
      if (h[6 + k])
        printf("  %s: %llu tasks, busy %.2f us, wait %.2f us per task\n", nm[k], h[6 + k],
               h[k] * 0.01 / h[6 + k], h[3 + k] * 0.01 / h[6 + k]);
  }
  printf("%s n=%u q=%llu batch=%zu io=%d: %.4f ms  %.2f Mpolymul/s  %.1f GB/s (%.1f%% of 8 TB/s)  chk=%016llx\n",
         VARIANT, n, (unsigned long long)q, batch, io_bits, ms, pps / 1e6, gbs, gbs / 80.0, sum);
  return 0;
}
