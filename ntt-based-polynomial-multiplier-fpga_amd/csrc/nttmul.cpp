// nttmul.cpp — host runtime behind include/nttmul.h (C ABI over the HIP runtime).
//
// Replaces the reference's host<->FPGA communicator one-for-one:
//   PCIE_Load/PCIE_Open (PCIE.c:59-103, NTT_PCIECommunicationv2.c:274)  -> nttmul_create
//   mode-0 DmaFifoWrite of W/W_INV/q/n_inv (NTT_PCIECommunicationv2.c:137-178)
//                                                                      -> table upload in create
//   mode-1/2 DmaFifoWrite(A/B) (:183-206)                              -> hipMemcpyAsync H2D
//   mode-3 SendCommand + WaitForDoneAll polling (:211-215, :83-107)   -> launch + stream sync
//   DmaFifoRead(C) (:220-224)                                          -> hipMemcpyAsync D2H
//   szError + goto cleanup / return FALSE (:175-178, :242-251)         -> negative status codes
// and provides the software path's entry points (ntt256_product1/4, NTT/ntt256.h:85-86) as
// compat shims.  There is no CPU fallback anywhere in this library.
#include <hip/hip_runtime.h>
#include <hsa/hsa_ext_amd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "copy_pool.hpp"
#include "launch.hpp"
#include "nttmul.h"

#include "planner.hpp"

using namespace nttmul;

namespace {

constexpr int kMaxDev = 16;
constexpr int kSlots = 3;                     // host-path pipeline depth per device
constexpr size_t kChunkBytes = 8u << 20;      // host-path chunk, per operand

// Multi-pass scratch (n > 4096: the column/row intermediates) and the bit-reversed copy of a
// reordered transform's input, sized for a sub-batch of at most params.scratch_mb per buffer.
// Every use is ordered after the previous one by `ev`, whatever stream it was enqueued on: two
// device-API calls on different streams (or two host-path slots) never overwrite each other's
// intermediates.
struct Scratch {
  void *buf[3] = {nullptr, nullptr, nullptr};
  size_t bytes = 0;
  void *perm = nullptr;
  size_t perm_bytes = 0;
  hipEvent_t ev = nullptr;                    // recorded after the last enqueued use
  bool used = false;
  hipStream_t last = nullptr;                 // stream of that use
};

struct DevState {
  int id = -1;
  hipStream_t stream = nullptr;
  void *fw = nullptr, *iw = nullptr;
  Scratch dscr;                               // device-resident API calls
  // host-buffer path: kSlots pipeline slots, each with a stream, pinned host staging, device
  // buffers for a, b, c and its own scratch (run_host)
  hipStream_t xs[kSlots] = {};
  void *pin[kSlots][3] = {};
  void *pin_dev[kSlots][3] = {};              // the same pinned buffers as device pointers
  void *dbuf[kSlots][3] = {};
  Scratch sscr[kSlots];
  size_t slot_bytes = 0;
  int *flag = nullptr;                        // range-check result
  int cus = 0;                                // compute units (persistent grid sizing)
  // stream of the last fused product launch (run_device).  A product launched on another
  // stream than the previous one keeps oldest-first issue (LaunchTables::prio_ok): launches on
  // alternating streams overlap, and oldest-first serves overlapping launches better.  (An event
  // query per call would say whether the previous launch still runs, but hipEventRecord +
  // hipEventQuery cost more host time per call than a C2 launch takes: 244 -> 218 M/s.)
  std::atomic<uintptr_t> prod_s{0};  // (uintptr_t)stream | 1 (the null stream is a stream too); 0: none
};

// The small-transaction device server (kernels.hip k_server): its mailbox (launch.hpp: the
// request half in host-mapped device memory, the result half in page-locked host memory) and the
// stream its resident kernel runs on.
struct Server {
  ServerReq *req = nullptr;                   // the request half as the host writes it
  ServerReq *dreq = nullptr;                  // ... as the kernel reads it
  bool req_in_vram = false;                   // (false: pinned host memory, req == host pointer)
  ServerBox *box = nullptr;
  ServerBox *dbox = nullptr;                  // the result half as a device pointer
  hipStream_t s = nullptr;
  unsigned seq = 0;                           // sequence number of the last go word posted
  unsigned served = 0;                        // the last go word whose product was received
  uint64_t host_ns = 0;                       // go -> done seen on the host, last request
  bool running = false;                       // launched and not known to have left
  std::chrono::steady_clock::time_point launched, last_done;
  // setup / launch failures (server_unavailable): how many, the last one's message, and how many
  // more eligible calls take the launch path before the server is tried again (advisor r5)
  unsigned failures = 0, cooldown = 0;
  char reason[192] = {0};
};
// The resident kernel occupies its hardware queue (4 per process on the box) while it waits, so
// work other streams place in that queue -- and a device-wide synchronize -- waits behind it.  It
// therefore stays only briefly: 1 ms without a request, 50 ms in all (then the next call
// relaunches it, ~20 us), and the context stops it before it enqueues any other work (advisor r4).
constexpr unsigned long long kServerIdleTicks = 100000;    // 1 ms at 100 MHz (s_memrealtime)
constexpr unsigned long long kServerLifeTicks = 5000000;   // 50 ms
constexpr auto kServerIdleHost = std::chrono::microseconds(500);  // host-side margins: past
constexpr auto kServerLifeHost = std::chrono::milliseconds(25);   // these, stop and relaunch

}  // namespace

struct nttmul_ctx {
  Plan plan;
  uint32_t flags = 0;
  int ndev = 0;
  DevState dev[kMaxDev];
  char err[256] = {0};
  // nttmul_params knobs, fixed at create (include/nttmul.h)
  int issue_prio = 0;                         // -1 never, 0 automatic, 1 always
  size_t zero_copy = 64u << 10;               // per-operand bytes run zero-copy (0: never)
  unsigned copy_threads = 8;
  size_t scratch_bytes = (size_t)512 << 20;   // per scratch buffer
  int small_server = 0;                       // 0 automatic, -1 never
  Server server;                              // on dev[0]
  int last_path = -1;                         // run_host: 0 staged, 1 direct DMA, 2 zero-copy
  // the last product launch (run_device, under g_err_mu): nttmul_last_kernel_name re-describes it
  struct {
    size_t batch = 0;
    int io_bits = 0, prio_ok = 1, dev = -1;
  } last_prod;
};

namespace {

// Restores the caller's current device on scope exit (torch and others rely on it).
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() { (void)hipGetDevice(&prev); }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// (the host-buffer path drives several devices from their own threads: one writer at a time)
std::mutex g_err_mu;

int fail(nttmul_ctx *ctx, hipError_t e, const char *what) {
  if (ctx) {
    std::lock_guard<std::mutex> l(g_err_mu);
    snprintf(ctx->err, sizeof(ctx->err), "%s: %s", what, hipGetErrorString(e));
  }
  return e == hipErrorOutOfMemory ? NTTMUL_ENOMEM : NTTMUL_EHIP;
}

// a status message of our own (same lock as fail)
void set_err(nttmul_ctx *ctx, const char *msg) {
  std::lock_guard<std::mutex> l(g_err_mu);
  snprintf(ctx->err, sizeof(ctx->err), "%s", msg);
}

#define HIP_TRY(ctx, expr)                          \
  do {                                              \
    hipError_t _e = (expr);                         \
    if (_e != hipSuccess) return fail(ctx, _e, #expr); \
  } while (0)

LaunchTables tables_for(const nttmul_ctx *ctx, const DevState &d) {
  const Plan &P = ctx->plan;
  LaunchTables T;
  T.logn = P.logn;
  T.word_bits = P.word_bits;
  T.q = P.q;
  T.qinv_neg = P.qinv_neg;
  T.f = P.f; T.fs = P.fs; T.wf = P.wf; T.wfs = P.wfs;
  T.f4 = P.f4; T.f4s = P.f4s; T.wf4 = P.wf4; T.wf4s = P.wf4s;
  T.f8 = P.f8; T.f8s = P.f8s; T.wf8 = P.wf8; T.wf8s = P.wf8s;
  T.fi = P.fi; T.fis = P.fis; T.wfi = P.wfi; T.wfis = P.wfis; T.r2 = P.r2;
  T.fw = d.fw;
  T.iw = d.iw;
  T.tw_bytes = P.fw.size();
  T.cus = d.cus;
  T.prio = ctx->issue_prio;
  return T;
}

DevState *find_dev(nttmul_ctx *ctx, int dev) {
  for (int i = 0; i < ctx->ndev; i++)
    if (ctx->dev[i].id == dev) return &ctx->dev[i];
  return nullptr;
}

// (Re)allocate nb buffers of at least `need` bytes; `sc`'s last use must have completed before
// the old ones are freed.
int ensure(nttmul_ctx *ctx, Scratch &sc, void **bufs, int nb, size_t *have, size_t need) {
  if (*have >= need) return NTTMUL_OK;
  if (sc.used) HIP_TRY(ctx, hipEventSynchronize(sc.ev));
  for (int i = 0; i < nb; i++) {
    if (bufs[i]) (void)hipFree(bufs[i]);
    bufs[i] = nullptr;
  }
  *have = 0;
  for (int i = 0; i < nb; i++) HIP_TRY(ctx, hipMalloc(&bufs[i], need));
  *have = need;
  return NTTMUL_OK;
}

// Polynomials per multi-pass / reordered-transform sub-batch: params.scratch_mb (default 512) MiB
// per scratch buffer (C5: the whole 1024-product batch in one pass).  Smaller sub-batches keep a
// sub-batch's intermediates in the 256 MiB Infinity Cache but cost more than they save: C5 at
// 8/16/32/64/128 MiB ran 2.86/1.91/1.60/1.48/1.40 ms against 1.36 ms in one pass
// (gpurun_out/r2a) — each sub-batch launch is a single generation of blocks.  The
// bound caps scratch memory for very large batches.
size_t sub_batch(const nttmul_ctx *ctx, size_t poly_bytes, size_t batch) {
  return std::max<size_t>(1, std::min(batch, ctx->scratch_bytes / poly_bytes));
}

int scratch_acquire(nttmul_ctx *ctx, Scratch &sc, hipStream_t s) {
  if (!sc.ev) HIP_TRY(ctx, hipEventCreateWithFlags(&sc.ev, hipEventDisableTiming));
  if (sc.used && sc.last != s) HIP_TRY(ctx, hipStreamWaitEvent(s, sc.ev, 0));
  return NTTMUL_OK;
}

int scratch_release(nttmul_ctx *ctx, Scratch &sc, hipStream_t s) {
  HIP_TRY(ctx, hipEventRecord(sc.ev, s));
  sc.used = true;
  sc.last = s;
  return NTTMUL_OK;
}

void scratch_free(Scratch &sc) {
  if (sc.used) (void)hipEventSynchronize(sc.ev);
  for (void *p : {sc.buf[0], sc.buf[1], sc.buf[2], sc.perm})
    if (p) (void)hipFree(p);
  if (sc.ev) (void)hipEventDestroy(sc.ev);
  sc = Scratch();
}

// Transforms are OP_XFORM + an NTTMUL_XF_* mode (direction | order | scaling).
enum Op {
  OP_MULTIPLY = 0,
  OP_POINTWISE = 3,
  OP_XFORM = 16,
  OP_FORWARD = OP_XFORM + (NTTMUL_XF_FORWARD | NTTMUL_XF_STD2REV),
  OP_INVERSE = OP_XFORM + (NTTMUL_XF_INVERSE | NTTMUL_XF_REV2STD),
};
constexpr unsigned kXfModes = NTTMUL_XF_INVERSE | NTTMUL_XF_REV2STD | NTTMUL_XF_UNSCALED;

void note_product(nttmul_ctx *ctx, const DevState &d, size_t batch, int io_bits, int prio_ok) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  ctx->last_prod.batch = batch;
  ctx->last_prod.io_bits = io_bits;
  ctx->last_prod.prio_ok = prio_ok;
  ctx->last_prod.dev = (int)(&d - ctx->dev);
}

// Enqueue one device-resident batch of `op` on d (current device must be d.id), using scratch sc
// where the op needs it.  b is unused by the transforms.
int run_device(nttmul_ctx *ctx, DevState &d, Scratch &sc, int op, void *c, const void *a,
               const void *b, size_t batch, int io_bits, hipStream_t s) {
  const Plan &P = ctx->plan;
  if (io_bits != 32 && io_bits != 64) return NTTMUL_EINVAL;
  if (io_bits == 32 && P.q > 0xFFFFFFFFull) return NTTMUL_EINVAL;  // q does not fit the words
  if (!batch) return NTTMUL_OK;  // an empty batch: nothing enqueued, no pointer dereferenced
  if (ctx->flags & NTTMUL_FLAG_VALIDATE) {
    HIP_TRY(ctx, hipMemsetAsync(d.flag, 0, sizeof(int), s));
    HIP_TRY(ctx, launch_check_range(a, (op == OP_MULTIPLY || op == OP_POINTWISE) ? b : a, P.q,
                                    batch * P.n, io_bits, d.flag, s));
    int bad = 0;
    HIP_TRY(ctx, hipMemcpyAsync(&bad, d.flag, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(ctx, hipStreamSynchronize(s));
    if (bad) {
      set_err(ctx, "input coefficient >= q");
      return NTTMUL_ERANGE;
    }
  }
  LaunchTables T = tables_for(ctx, d);
  const size_t io_poly = (size_t)P.n * (io_bits / 8), w_poly = (size_t)P.n * (P.word_bits / 8);
  bool inv = false, reorder = false;
  if (op >= OP_XFORM) {
    const unsigned mode = (unsigned)(op - OP_XFORM);
    if (mode & ~kXfModes) return NTTMUL_EINVAL;
    inv = mode & NTTMUL_XF_INVERSE;
    // the kernels run forward std2rev and inverse rev2std; the other orders are the same
    // transform between two bit-reversal permutations (rev2std = P o std2rev o P, verified on
    // the reference's own loops: tests/golden/ref256_wrappers.npz)
    reorder = inv != ((mode & NTTMUL_XF_REV2STD) != 0);
    if (mode & NTTMUL_XF_UNSCALED) {
      if (!inv) return NTTMUL_EINVAL;
      T.fi = P.fu; T.fis = P.fus; T.wfi = P.wfu; T.wfis = P.wfus;
    }
  } else if (op != OP_MULTIPLY && op != OP_POINTWISE) {
    return NTTMUL_EINVAL;
  }
  const bool multipass = P.logn > 12 && op != OP_POINTWISE;
  if (!multipass && !reorder) {  // one launch over the whole batch, no scratch
    if (op == OP_MULTIPLY) {
      const uintptr_t tag = (uintptr_t)s | 1;
      const uintptr_t prev = d.prod_s.exchange(tag, std::memory_order_relaxed);
      if (prev && prev != tag) T.prio_ok = 0;
      HIP_TRY(ctx, launch_polymul(T, a, b, c, batch, io_bits, sc.buf, s));
      note_product(ctx, d, batch, io_bits, T.prio_ok);
      return NTTMUL_OK;
    }
    else if (op == OP_POINTWISE) HIP_TRY(ctx, launch_pointwise(T, a, b, c, batch, io_bits, s));
    else HIP_TRY(ctx, launch_xform(T, a, c, batch, io_bits, inv, sc.buf, s));
    return NTTMUL_OK;
  }
  // sub-batches through the scratch
  const size_t chunk = sub_batch(ctx, multipass ? w_poly : io_poly, batch);
  int st = scratch_acquire(ctx, sc, s);
  if (st) return st;
  if (multipass && (st = ensure(ctx, sc, sc.buf, 3, &sc.bytes, chunk * w_poly))) return st;
  if (reorder && (st = ensure(ctx, sc, &sc.perm, 1, &sc.perm_bytes, chunk * io_poly))) return st;
  for (size_t p = 0; p < batch && !st; p += chunk) {
    const size_t cnt = std::min(chunk, batch - p);
    const char *ap = (const char *)a + p * io_poly;
    const char *bp = b ? (const char *)b + p * io_poly : nullptr;
    char *cp = (char *)c + p * io_poly;
    hipError_t e;
    if (op == OP_MULTIPLY) {
      e = launch_polymul(T, ap, bp, cp, cnt, io_bits, sc.buf, s);
    } else if (!reorder) {
      e = launch_xform(T, ap, cp, cnt, io_bits, inv, sc.buf, s);
    } else if ((e = launch_bitrev(ap, sc.perm, P.logn, cnt, io_bits, s)) == hipSuccess &&
               (e = launch_xform(T, sc.perm, cp, cnt, io_bits, inv, sc.buf, s)) == hipSuccess) {
      e = launch_bitrev(cp, cp, P.logn, cnt, io_bits, s);
    }
    if (e != hipSuccess) st = fail(ctx, e, "sub-batch launch");
  }
  if (!st && op == OP_MULTIPLY) note_product(ctx, d, chunk, io_bits, T.prio_ok);
  const int rel = scratch_release(ctx, sc, s);
  return st ? st : rel;
}

void pcopy(const nttmul_ctx *ctx, void *dst, const void *src, size_t bytes) {
  CopyPool::get().copy(dst, src, bytes, ctx->copy_threads);
}

int ensure_slots(nttmul_ctx *ctx, DevState &d, size_t bytes) {
  for (int s = 0; s < kSlots; s++)
    if (!d.xs[s]) HIP_TRY(ctx, hipStreamCreateWithFlags(&d.xs[s], hipStreamNonBlocking));
  if (d.slot_bytes >= bytes) return NTTMUL_OK;
  for (int s = 0; s < kSlots; s++) {
    HIP_TRY(ctx, hipStreamSynchronize(d.xs[s]));
    for (int k = 0; k < 3; k++) {
      if (d.pin[s][k]) (void)hipHostFree(d.pin[s][k]);
      if (d.dbuf[s][k]) (void)hipFree(d.dbuf[s][k]);
      d.pin[s][k] = d.pin_dev[s][k] = d.dbuf[s][k] = nullptr;
    }
  }
  d.slot_bytes = 0;
  for (int s = 0; s < kSlots; s++)
    for (int k = 0; k < 3; k++) {
      HIP_TRY(ctx, hipHostMalloc(&d.pin[s][k], bytes, hipHostMallocDefault));
      HIP_TRY(ctx, hipHostGetDevicePointer(&d.pin_dev[s][k], d.pin[s][k], 0));
      HIP_TRY(ctx, hipMalloc(&d.dbuf[s][k], bytes));
    }
  d.slot_bytes = bytes;
  return NTTMUL_OK;
}

// True when [p, p + bytes) lies inside ONE page-locked host allocation the copy engines can DMA
// directly (hipHostMalloc'd or hipHostRegister'ed): the allocation that holds p (its device
// view's address range) must also hold p + bytes - 1.  Anything else — pageable memory, a range
// spanning two pinned blocks or pageable memory between two pinned ends — takes the staged path.
bool host_pinned(const void *p, size_t bytes) {
  if (!p || !bytes) return false;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: the query fails, clear the sticky error
    return false;
  }
  if (at.type != hipMemoryTypeHost || !at.devicePointer) return false;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)at.devicePointer) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  const char *d0 = (const char *)at.devicePointer, *b0 = (const char *)base;
  return d0 >= b0 && (size_t)(d0 - b0) <= size && bytes <= size - (size_t)(d0 - b0);
}

// Host-buffer path (the FPGA transaction: mode 1/2 DMA in, mode 3, DMA out).  Each device's
// contiguous slice [p0, p1) streams through kSlots pipeline slots in chunks: the host
// copies chunk j into pinned staging while the GPU runs H2D -> kernel -> D2H of chunks j-1, j-2 on
// the other slots' streams, and copies a finished chunk's result out when its slot comes round
// again.  `direct`: a, b, c are page-locked, so the copy engines DMA each chunk straight from and
// to them and the host only waits at the end.
struct HostJob {
  int op, io_bits;
  void *c;
  const void *a, *b;
  size_t pbytes, chunk, zero_copy;
  bool direct;
};

int run_host_dev(nttmul_ctx *ctx, DevState &d, const HostJob &J, size_t p0, size_t p1) {
  const bool two = J.op == OP_MULTIPLY || J.op == OP_POINTWISE;
  struct Pending {
    bool busy = false;
    size_t off = 0, bytes = 0;
  } slot[kSlots];
  HIP_TRY(ctx, hipSetDevice(d.id));
  int st = ensure_slots(ctx, d, std::min(J.chunk, p1 - p0) * J.pbytes);
  if (st) return st;
  auto retire = [&](int s) -> int {
    Pending &pd = slot[s];
    if (!pd.busy) return NTTMUL_OK;
    pd.busy = false;
    HIP_TRY(ctx, hipStreamSynchronize(d.xs[s]));
    if (!J.direct) pcopy(ctx, (char *)J.c + pd.off, d.pin[s][2], pd.bytes);
    return NTTMUL_OK;
  };
  unsigned k = 0;
  for (size_t next = p0; next < p1 && !st;) {
    const int s = (int)(k++ % kSlots);
    const size_t cnt = std::min(J.chunk, p1 - next);
    const size_t off = next * J.pbytes, bytes = cnt * J.pbytes;
    hipError_t e = hipSuccess;
    if (J.direct) {
      e = hipMemcpyAsync(d.dbuf[s][0], (const char *)J.a + off, bytes, hipMemcpyHostToDevice,
                         d.xs[s]);
      if (e == hipSuccess && two)
        e = hipMemcpyAsync(d.dbuf[s][1], (const char *)J.b + off, bytes, hipMemcpyHostToDevice,
                           d.xs[s]);
      if (e != hipSuccess) { st = fail(ctx, e, "hipMemcpyAsync H2D"); break; }
      if ((st = run_device(ctx, d, d.sscr[s], J.op, d.dbuf[s][2], d.dbuf[s][0], d.dbuf[s][1],
                           cnt, J.io_bits, d.xs[s])))
        break;
      e = hipMemcpyAsync((char *)J.c + off, d.dbuf[s][2], bytes, hipMemcpyDeviceToHost, d.xs[s]);
      if (e != hipSuccess) { st = fail(ctx, e, "hipMemcpyAsync D2H"); break; }
      slot[s] = Pending{true, off, bytes};
      next += cnt;
      continue;
    }
    if ((st = retire(s))) break;
    pcopy(ctx, d.pin[s][0], (const char *)J.a + off, bytes);
    if (two) pcopy(ctx, d.pin[s][1], (const char *)J.b + off, bytes);
    if (bytes <= J.zero_copy && ctx->plan.logn <= 12) {
      // small transaction (the ntt256_product* shims): the kernel reads a, b from and writes c to
      // the pinned staging buffers over PCIe — no copy-engine round trips
      if ((st = run_device(ctx, d, d.sscr[s], J.op, d.pin_dev[s][2], d.pin_dev[s][0],
                           d.pin_dev[s][1], cnt, J.io_bits, d.xs[s])))
        break;
      slot[s] = Pending{true, off, bytes};
      next += cnt;
      continue;
    }
    e = hipMemcpyAsync(d.dbuf[s][0], d.pin[s][0], bytes, hipMemcpyHostToDevice, d.xs[s]);
    if (e == hipSuccess && two)
      e = hipMemcpyAsync(d.dbuf[s][1], d.pin[s][1], bytes, hipMemcpyHostToDevice, d.xs[s]);
    if (e != hipSuccess) { st = fail(ctx, e, "hipMemcpyAsync H2D"); break; }
    if ((st = run_device(ctx, d, d.sscr[s], J.op, d.dbuf[s][2], d.dbuf[s][0], d.dbuf[s][1], cnt,
                         J.io_bits, d.xs[s])))
      break;
    e = hipMemcpyAsync(d.pin[s][2], d.dbuf[s][2], bytes, hipMemcpyDeviceToHost, d.xs[s]);
    if (e != hipSuccess) { st = fail(ctx, e, "hipMemcpyAsync D2H"); break; }
    slot[s] = Pending{true, off, bytes};
    next += cnt;
  }
  // drain (also after an error, so no slot is left in flight and no DMA still touches the
  // caller's buffers when the call returns)
  for (int s = 0; s < kSlots; s++) {
    const int r = retire(s);
    if (!st) st = r;
  }
  return st;
}

// Small host transactions (params.small_server; kernels.hip k_server): the FPGA flow's mode 3 +
// WaitForDoneAll (NTT_PCIECommunicationv2.c:83-107, 211-215) without a kernel launch per call.
// The caller's a, b go into the mailbox, go = seq releases them, and the host spins on done;
// the resident kernel is (re)launched when it is not known to be alive: never launched, idle on
// the host's clock for longer than kServerIdleHost (it leaves after 1 ms on its own), older than
// kServerLifeHost, or found finished while a request waits.  Every spin is bounded.
// The go word into the request half.  A BAR mapping of device memory is uncached or
// write-combining on the host, so the fences keep a and b ahead of go and push go out at once.
void post_go(Server &S, unsigned v) {
  __builtin_ia32_sfence();
  __atomic_store_n(&S.req->go, v, __ATOMIC_RELEASE);
  __builtin_ia32_sfence();
}

int server_stop(nttmul_ctx *ctx) {
  Server &S = ctx->server;
  if (!S.running) return NTTMUL_OK;
  // a stop request: a new sequence number with count 0
  post_go(S, ((++S.seq) << 8) | ServerBox::kStop);
  S.running = false;
  const hipError_t e = hipStreamSynchronize(S.s);
  // (the stop needs no answer: a relaunched kernel starts from done = S.served, and the next
  // request's go differs from both)
  post_go(S, S.served);
  return e == hipSuccess ? NTTMUL_OK : fail(ctx, e, "device server exit");
}

int server_launch(nttmul_ctx *ctx, DevState &d) {
  Server &S = ctx->server;
  // the kernel starts from done: the last request it must not serve again (no kernel runs now)
  __atomic_store_n(&S.box->done, S.served, __ATOMIC_RELEASE);
  DeviceGuard guard;
  HIP_TRY(ctx, hipSetDevice(d.id));
  HIP_TRY(ctx, launch_server(tables_for(ctx, d), S.dreq, S.dbox, kServerIdleTicks,
                             kServerLifeTicks, S.s));
  S.running = true;
  S.launched = S.last_done = std::chrono::steady_clock::now();
  return NTTMUL_OK;
}

// The mailbox (launch.hpp ServerReq / ServerBox).  The request half goes to fine-grained device
// memory when the runtime gives the host a mapping of it (large BAR) and a probe written through
// that mapping reads back through the device; otherwise to pinned host memory.
int server_alloc(nttmul_ctx *ctx, DevState &d) {
  Server &S = ctx->server;
  DeviceGuard guard;
  HIP_TRY(ctx, hipSetDevice(d.id));
  if (!S.box) {
    HIP_TRY(ctx, hipHostMalloc((void **)&S.box, sizeof(ServerBox), hipHostMallocCoherent));
    memset((void *)S.box, 0, sizeof(ServerBox));
    HIP_TRY(ctx, hipHostGetDevicePointer((void **)&S.dbox, S.box, 0));
  }
  if (!S.s) HIP_TRY(ctx, hipStreamCreateWithFlags(&S.s, hipStreamNonBlocking));
  void *dv = nullptr;
  if (hipExtMallocWithFlags(&dv, sizeof(ServerReq), hipDeviceMallocFinegrained) == hipSuccess) {
    hsa_amd_pointer_info_t info;
    memset(&info, 0, sizeof(info));
    info.size = sizeof(info);
    ServerReq *hv = nullptr;
    if (hsa_amd_pointer_info(dv, &info, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
        info.hostBaseAddress && info.agentBaseAddress) {  // (dv may lie inside a larger block)
      const size_t off = (size_t)((char *)dv - (char *)info.agentBaseAddress);
      if (off + sizeof(ServerReq) <= info.sizeInBytes)
        hv = (ServerReq *)((char *)info.hostBaseAddress + off);
    }
    uint32_t back = 0;
    if (hv) {
      __atomic_store_n(&hv->go, 0x5A5A5A5Au, __ATOMIC_RELEASE);
      __builtin_ia32_sfence();
      if (hipMemcpy(&back, &((ServerReq *)dv)->go, 4, hipMemcpyDeviceToHost) != hipSuccess) back = 0;
    }
    if (back == 0x5A5A5A5Au) {
      S.req = hv;
      S.dreq = (ServerReq *)dv;
      S.req_in_vram = true;
    } else {
      (void)hipFree(dv);
    }
  }
  (void)hipGetLastError();
  if (!S.req) {
    HIP_TRY(ctx, hipHostMalloc((void **)&S.req, sizeof(ServerReq), hipHostMallocCoherent));
    HIP_TRY(ctx, hipHostGetDevicePointer((void **)&S.dreq, S.req, 0));
  }
  post_go(S, 0);
  return NTTMUL_OK;
}

// The context's server leaves before the context enqueues anything else (run_device, the launch
// path of run_host, fills): its kernel would otherwise hold that work's hardware queue until its
// idle exit.
int server_quiesce(nttmul_ctx *ctx) { return ctx->server.running ? server_stop(ctx) : NTTMUL_OK; }

// The server could not be set up or launched (status st: the runtime refused an allocation,
// a launch, ...): this call takes the launch path.  The failure is kept for nttmul_server_status
// (count and message) instead of vanishing with the cleared error string: an out-of-memory
// failure retries the server after the next 64 eligible calls, up to 3 failures in all; any other
// failure, or the third, leaves the launch path for the context's lifetime.
constexpr unsigned kServerRetryCalls = 64, kServerMaxFailures = 3;
int server_unavailable(nttmul_ctx *ctx, int st) {
  Server &S = ctx->server;
  S.running = false;
  (void)hipGetLastError();
  S.failures++;
  const bool retry = st == NTTMUL_ENOMEM && S.failures < kServerMaxFailures;
  {
    std::lock_guard<std::mutex> l(g_err_mu);
    char msg[sizeof(ctx->err)];
    snprintf(msg, sizeof(msg), "%s", ctx->err);
    if (retry)
      snprintf(S.reason, sizeof(S.reason), "failure %u (%s): %s; retried after %u calls", S.failures,
               nttmul_strerror(st), msg, kServerRetryCalls);
    else
      snprintf(S.reason, sizeof(S.reason), "failure %u (%s): %s; launch path from now on",
               S.failures, nttmul_strerror(st), msg);
    ctx->err[0] = 0;  // (the call itself succeeds on the launch path)
  }
  if (retry)
    S.cooldown = kServerRetryCalls;
  else
    ctx->small_server = -1;
  return 1;
}

// >0: not served here (the caller takes the launch path); else a status
int run_server(nttmul_ctx *ctx, void *c, const void *a, const void *b, size_t batch) {
  const Plan &P = ctx->plan;
  const size_t words = batch * P.n;
  if (ctx->small_server < 0 || ctx->ndev != 1 || P.word_bits != 32 || P.logn < 8 || P.logn > 10 ||
      words > (size_t)ServerBox::kWords || a32_kind(P.q) != A32Kind::Plantard ||
      P.fw.size() / 8 > P.n)  // (launch_server copies n twiddle pairs of 2 x u32 into LDS)
    return 1;
  if (ctx->flags & NTTMUL_FLAG_VALIDATE) {  // the range check of run_device, on the host
    const uint32_t *pa = (const uint32_t *)a, *pb = (const uint32_t *)b;
    for (size_t i = 0; i < words; i++)
      if (pa[i] >= P.q || pb[i] >= P.q) {
        set_err(ctx, "input coefficient >= q");
        return NTTMUL_ERANGE;
      }
  }
  Server &S = ctx->server;
  if (S.cooldown) {  // after a transient setup failure (server_unavailable)
    S.cooldown--;
    return 1;
  }
  DevState &d = ctx->dev[0];
  if (!S.req) {
    const int st = server_alloc(ctx, d);
    if (st) return server_unavailable(ctx, st);
  }
  const auto now = std::chrono::steady_clock::now();
  if (S.running && (now - S.last_done > kServerIdleHost || now - S.launched > kServerLifeHost)) {
    const int st = server_stop(ctx);
    if (st) return st;
  }
  if (!S.running) {
    const int st = server_launch(ctx, d);
    if (st) return server_unavailable(ctx, st);
  }
  // Completion is the result itself: c is set to a word no product can hold (the server's
  // q < 2^31, so 0xFFFFFFFF) before go, and the request is done when no word of c still holds it.
  // Every 4-byte store of the kernel lands whole, so this needs no release fence and no done word
  // on the device side (one PCIe write round trip less per request).
  uint32_t *bc = S.box->c;
  for (size_t i = 0; i < words; i++) bc[i] = ServerBox::kPending;
  memcpy(S.req->a, a, words * 4);
  memcpy(S.req->b, b, words * 4);
  const unsigned seq = ((++S.seq) << 8) | (unsigned)batch;  // batch <= 4: one go word
  const auto t0 = std::chrono::steady_clock::now();
  post_go(S, seq);
  const auto landed = [&]() {
    for (size_t i = 0; i < words; i++)
      if (__atomic_load_n(bc + i, __ATOMIC_RELAXED) == ServerBox::kPending) return false;
    std::atomic_thread_fence(std::memory_order_acquire);
#ifdef NTTMUL_CLOCK_STAMPS  // (the diagnostic build's stamps are released with done)
    if (__atomic_load_n(&S.box->done, __ATOMIC_ACQUIRE) != seq) return false;
#endif
    return true;
  };
  for (unsigned spin = 1; !landed(); spin++) {
    __builtin_ia32_pause();
    if (spin % 1024) continue;
    const hipError_t q = hipStreamQuery(S.s);
    if (q == hipSuccess) {
      // the kernel has left, and a finished kernel's stores have all landed: either it served
      // this request after the check above, or it left before it saw it -- then relaunch
      if (landed()) break;
      S.running = false;
      // (a relaunch the runtime refuses: this request takes the launch path)
      const int st = server_launch(ctx, d);
      if (st) return server_unavailable(ctx, st);
    } else if (q != hipErrorNotReady) {
      S.running = false;
      return fail(ctx, q, "device server");
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
      (void)server_stop(ctx);
      set_err(ctx, "device server: no answer within 5 s");
      return NTTMUL_EHIP;
    }
  }
  S.served = seq;
  S.last_done = std::chrono::steady_clock::now();
  S.host_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(S.last_done - t0).count();
  memcpy(c, bc, words * 4);
  ctx->last_path = 3;
  return NTTMUL_OK;
}

// The batch splits into one contiguous slice per context device; with several devices each slice
// is driven by its own host thread (slice 0 by the caller's), so one device's staging copies and
// synchronisations never stall another's pipeline.
int run_host(nttmul_ctx *ctx, int op, void *c, const void *a, const void *b, size_t batch,
             int io_bits) {
  const bool two = op == OP_MULTIPLY || op == OP_POINTWISE;
  // pointers may be null for an empty batch, as on the device path (device_op)
  if (!ctx || (batch && (!c || !a || (two && !b)))) return NTTMUL_EINVAL;
  if (io_bits != 32 && io_bits != 64) return NTTMUL_EINVAL;
  if (io_bits == 32 && ctx->plan.q > 0xFFFFFFFFull) return NTTMUL_EINVAL;
  if (!batch) return NTTMUL_OK;
  if (op == OP_MULTIPLY && io_bits == 32) {  // (no HIP call on the server's fast path)
    const int st = run_server(ctx, c, a, b, batch);
    if (st <= 0) return st;
  }
  if (const int st = server_quiesce(ctx)) return st;
  DeviceGuard guard;
  HostJob J;
  J.op = op;
  J.io_bits = io_bits;
  J.c = c;
  J.a = a;
  J.b = b;
  J.pbytes = (size_t)ctx->plan.n * (io_bits / 8);
  J.chunk = std::max<size_t>(1, kChunkBytes / J.pbytes);
  // per-operand bytes up to which a chunk runs zero-copy on the pinned staging buffers
  // (params.zero_copy_kb)
  J.zero_copy = ctx->zero_copy;
  const size_t total = batch * J.pbytes;
  J.direct = host_pinned(a, total) && (!two || host_pinned(b, total)) && host_pinned(c, total);
  const size_t first_chunk = std::min(J.chunk, std::max<size_t>(1, batch / ctx->ndev));
  ctx->last_path = J.direct ? 1 : (first_chunk * J.pbytes <= J.zero_copy &&
                                   ctx->plan.logn <= 12) ? 2 : 0;
  int status[kMaxDev] = {};
  std::vector<std::thread> th;
  for (int i = 1; i < ctx->ndev; i++) {
    const size_t p0 = batch * (size_t)i / ctx->ndev, p1 = batch * (size_t)(i + 1) / ctx->ndev;
    if (p1 <= p0) continue;
    try {
      th.emplace_back([ctx, &J, &status, i, p0, p1] {
        status[i] = run_host_dev(ctx, ctx->dev[i], J, p0, p1);
      });
    } catch (...) {  // no thread available: this slice runs on the caller's thread
      status[i] = run_host_dev(ctx, ctx->dev[i], J, p0, p1);
    }
  }
  const size_t p1 = batch / ctx->ndev;
  if (p1 > 0) status[0] = run_host_dev(ctx, ctx->dev[0], J, 0, p1);
  for (std::thread &t : th) t.join();
  for (int i = 0; i < ctx->ndev; i++)
    if (status[i]) return status[i];
  return NTTMUL_OK;
}

}  // namespace

extern "C" {

const char *nttmul_strerror(int status) {
  switch (status) {
    case NTTMUL_OK: return "ok";
    case NTTMUL_EINVAL: return "invalid argument (n, q, psi, word size or pointer)";
    case NTTMUL_ENODEV: return "no usable HIP device";
    case NTTMUL_EHIP: return "HIP runtime error";
    case NTTMUL_ENOMEM: return "out of memory";
    case NTTMUL_ERANGE: return "input coefficient out of range [0, q)";
    case NTTMUL_EUNSUPPORTED: return "unsupported parameter combination";
    default: return "unknown status";
  }
}

const char *nttmul_last_error(const nttmul_ctx *ctx) { return ctx ? ctx->err : ""; }

int nttmul_host_alloc(void **p, size_t bytes) {
  if (!p) return NTTMUL_EINVAL;
  *p = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    (void)hipGetLastError();
    return NTTMUL_ENODEV;
  }
  if (hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocPortable) != hipSuccess) {
    (void)hipGetLastError();
    *p = nullptr;
    return NTTMUL_ENOMEM;
  }
  return NTTMUL_OK;
}

void nttmul_host_free(void *p) {
  if (p) (void)hipHostFree(p);
}

// The struct's size is the caller's (advisor r4): a binary built against the round 1-3 header
// passes the six-field layout, whose knobs then take their defaults instead of being read from
// memory past the caller's struct.
int nttmul_create_sized(nttmul_ctx **out, const nttmul_params *caller, size_t size) {
  if (!out) return NTTMUL_EINVAL;
  *out = nullptr;
  if (!caller || size < NTTMUL_PARAMS_BASE_SIZE || size > sizeof(nttmul_params))
    return NTTMUL_EINVAL;
  nttmul_params p;
  memset(&p, 0, sizeof(p));
  memcpy(&p, caller, size);
  const nttmul_params *prm = &p;
  nttmul_ctx *ctx = new (std::nothrow) nttmul_ctx();
  if (!ctx) return NTTMUL_ENOMEM;
  int st = make_plan(prm->n, prm->q, prm->psi, &ctx->plan, (prm->flags & NTTMUL_FLAG_CYCLIC) != 0);
  if (st) {
    delete ctx;
    return st;
  }
  ctx->flags = prm->flags;
  if (prm->issue_prio < -1 || prm->issue_prio > 1 || prm->zero_copy_kb < -1 ||
      prm->copy_threads < 0) {
    delete ctx;
    return NTTMUL_EINVAL;
  }
  ctx->issue_prio = prm->issue_prio;
  ctx->zero_copy = prm->zero_copy_kb < 0 ? 0 : (size_t)(prm->zero_copy_kb ? prm->zero_copy_kb : 64) << 10;
  ctx->copy_threads = prm->copy_threads ? (unsigned)prm->copy_threads : 8u;
  ctx->scratch_bytes = (size_t)(prm->scratch_mb ? prm->scratch_mb : 512) << 20;
  if (prm->small_server < -1 || prm->small_server > 0) {
    delete ctx;
    return NTTMUL_EINVAL;
  }
  ctx->small_server = prm->small_server;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    delete ctx;
    return NTTMUL_ENODEV;
  }
  const int first = prm->first_dev < 0 ? 0 : prm->first_dev;
  int ndev = prm->ndev <= 0 ? count - first : prm->ndev;
  // NTTMUL_FLAG_SHARE_DEVICES: ndev slices over the devices first .. count - 1 round-robin (as
  // bench.py maps ranks), so the multi-device split also runs on a single GPU
  const bool share = (prm->flags & NTTMUL_FLAG_SHARE_DEVICES) != 0;
  if (first >= count || ndev <= 0 || (!share && first + ndev > count) || ndev > kMaxDev) {
    delete ctx;
    return NTTMUL_ENODEV;
  }
  DeviceGuard guard;
  const size_t tbytes = ctx->plan.fw.size();
  for (int i = 0; i < ndev; i++) {
    DevState &d = ctx->dev[i];
    d.id = first + i % (count - first);
    ctx->ndev = i + 1;
    hipError_t e;
    if ((e = hipSetDevice(d.id)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipMalloc(&d.fw, tbytes)) != hipSuccess || (e = hipMalloc(&d.iw, tbytes)) != hipSuccess ||
        (e = hipMalloc((void **)&d.flag, sizeof(int))) != hipSuccess ||
        (e = hipMemcpy(d.fw, ctx->plan.fw.data(), tbytes, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(d.iw, ctx->plan.iw.data(), tbytes, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipDeviceGetAttribute(&d.cus, hipDeviceAttributeMultiprocessorCount, d.id)) !=
            hipSuccess) {
      st = fail(ctx, e, "nttmul_create device setup");
      fprintf(stderr, "nttmul: %s\n", ctx->err);
      nttmul_destroy(ctx);
      return st == NTTMUL_EHIP ? NTTMUL_ENODEV : st;
    }
  }
  *out = ctx;
  return NTTMUL_OK;
}

int nttmul_create_ex(nttmul_ctx **ctx, const nttmul_params *prm) {
  return nttmul_create_sized(ctx, prm, NTTMUL_PARAMS_BASE_SIZE);
}

int nttmul_create(nttmul_ctx **ctx, uint32_t n, uint64_t q, int ndev) {
  nttmul_params p;
  memset(&p, 0, sizeof(p));
  p.n = n;
  p.q = q;
  p.ndev = ndev;
  return nttmul_create_ex(ctx, &p);
}

void nttmul_destroy(nttmul_ctx *ctx) {
  if (!ctx) return;
  DeviceGuard guard;
  Server &S = ctx->server;
  if (S.box || S.req || S.s) {  // whatever a partial server_alloc left behind
    (void)hipSetDevice(ctx->dev[0].id);
    (void)server_stop(ctx);
    if (S.s) (void)hipStreamDestroy(S.s);
    if (S.box) (void)hipHostFree(S.box);
    if (S.req_in_vram)
      (void)hipFree(S.dreq);
    else if (S.req)
      (void)hipHostFree(S.req);
  }
  for (int i = 0; i < ctx->ndev; i++) {
    DevState &d = ctx->dev[i];
    if (d.id < 0) continue;
    (void)hipSetDevice(d.id);
    if (d.stream) (void)hipStreamSynchronize(d.stream);
    for (int k = 0; k < kSlots; k++) {
      if (d.xs[k]) (void)hipStreamSynchronize(d.xs[k]);
      for (int m = 0; m < 3; m++) {
        if (d.pin[k][m]) (void)hipHostFree(d.pin[k][m]);
        if (d.dbuf[k][m]) (void)hipFree(d.dbuf[k][m]);
      }
      scratch_free(d.sscr[k]);
      if (d.xs[k]) (void)hipStreamDestroy(d.xs[k]);
    }
    scratch_free(d.dscr);
    for (void *p : {d.fw, d.iw, (void *)d.flag})
      if (p) (void)hipFree(p);
    if (d.stream) (void)hipStreamDestroy(d.stream);
  }
  delete ctx;
}

int nttmul_get_info(const nttmul_ctx *ctx, nttmul_info *info) {
  if (!ctx || !info) return NTTMUL_EINVAL;
  const Plan &P = ctx->plan;
  info->n = P.n;
  info->logn = P.logn;
  info->q = P.q;
  info->psi = P.psi;
  info->omega = P.omega;
  info->inv_psi = P.inv_psi;
  info->inv_omega = P.inv_omega;
  info->inv_n = P.inv_n;
  info->word_bits = (uint32_t)P.word_bits;
  info->ndev = ctx->ndev;
  info->kernel = P.logn > 12 ? 2 : 1;
  info->cyclic = P.cyclic ? 1 : 0;
  return NTTMUL_OK;
}

int nttmul_last_host_path(const nttmul_ctx *ctx) { return ctx ? ctx->last_path : NTTMUL_EINVAL; }

int nttmul_server_status(const nttmul_ctx *ctx, char *reason, size_t cap) {
  if (!ctx) return NTTMUL_EINVAL;
  if (reason && cap) snprintf(reason, cap, "%s", ctx->server.reason);
  return (int)ctx->server.failures;
}

int nttmul_kernel_name_batch(const nttmul_ctx *ctx, int word_bits, size_t batch, char *buf,
                             size_t cap) {
  if (!ctx || (word_bits != 32 && word_bits != 64) || (cap && !buf)) return NTTMUL_EINVAL;
  if (word_bits == 32 && ctx->plan.q > 0xFFFFFFFFull) return NTTMUL_EINVAL;
  std::string name;
  if (describe_polymul(tables_for(ctx, ctx->dev[0]), word_bits, batch, &name) != hipSuccess)
    return NTTMUL_EUNSUPPORTED;
  if (cap) {
    const size_t k = std::min(cap - 1, name.size());
    memcpy(buf, name.data(), k);
    buf[k] = 0;
  }
  return (int)name.size();
}
int nttmul_kernel_name(const nttmul_ctx *ctx, int word_bits, char *buf, size_t cap) {
  return nttmul_kernel_name_batch(ctx, word_bits, 0, buf, cap);
}

int nttmul_last_kernel_name(const nttmul_ctx *ctx, char *buf, size_t cap) {
  if (!ctx || (cap && !buf)) return NTTMUL_EINVAL;
  size_t batch;
  int io_bits, prio_ok, dev;
  {
    std::lock_guard<std::mutex> lk(g_err_mu);
    batch = ctx->last_prod.batch;
    io_bits = ctx->last_prod.io_bits;
    prio_ok = ctx->last_prod.prio_ok;
    dev = ctx->last_prod.dev;
  }
  std::string name;
  if (dev >= 0) {
    LaunchTables T = tables_for(ctx, ctx->dev[dev]);
    T.prio_ok = prio_ok;
    if (describe_polymul(T, io_bits, batch, &name) != hipSuccess) return NTTMUL_EUNSUPPORTED;
  }
  if (cap) {
    const size_t k = std::min(cap - 1, name.size());
    memcpy(buf, name.data(), k);
    buf[k] = 0;
  }
  return (int)name.size();
}

int nttmul_multiply_batch_u32(nttmul_ctx *ctx, uint32_t *c, const uint32_t *a, const uint32_t *b,
                              size_t batch) {
  return run_host(ctx, OP_MULTIPLY, c, a, b, batch, 32);
}
int nttmul_multiply_batch_u64(nttmul_ctx *ctx, uint64_t *c, const uint64_t *a, const uint64_t *b,
                              size_t batch) {
  return run_host(ctx, OP_MULTIPLY, c, a, b, batch, 64);
}
int nttmul_multiply_u32(nttmul_ctx *ctx, uint32_t *c, const uint32_t *a, const uint32_t *b) {
  return run_host(ctx, OP_MULTIPLY, c, a, b, 1, 32);
}
int nttmul_multiply_u64(nttmul_ctx *ctx, uint64_t *c, const uint64_t *a, const uint64_t *b) {
  return run_host(ctx, OP_MULTIPLY, c, a, b, 1, 64);
}
int nttmul_forward_batch_u32(nttmul_ctx *ctx, uint32_t *out, const uint32_t *in, size_t batch) {
  return run_host(ctx, OP_FORWARD, out, in, nullptr, batch, 32);
}
int nttmul_forward_batch_u64(nttmul_ctx *ctx, uint64_t *out, const uint64_t *in, size_t batch) {
  return run_host(ctx, OP_FORWARD, out, in, nullptr, batch, 64);
}
int nttmul_inverse_batch_u32(nttmul_ctx *ctx, uint32_t *out, const uint32_t *in, size_t batch) {
  return run_host(ctx, OP_INVERSE, out, in, nullptr, batch, 32);
}
int nttmul_inverse_batch_u64(nttmul_ctx *ctx, uint64_t *out, const uint64_t *in, size_t batch) {
  return run_host(ctx, OP_INVERSE, out, in, nullptr, batch, 64);
}
int nttmul_transform_batch_u32(nttmul_ctx *ctx, unsigned mode, uint32_t *out, const uint32_t *in,
                               size_t batch) {
  if (mode & ~kXfModes) return NTTMUL_EINVAL;
  return run_host(ctx, OP_XFORM + (int)mode, out, in, nullptr, batch, 32);
}
int nttmul_transform_batch_u64(nttmul_ctx *ctx, unsigned mode, uint64_t *out, const uint64_t *in,
                               size_t batch) {
  if (mode & ~kXfModes) return NTTMUL_EINVAL;
  return run_host(ctx, OP_XFORM + (int)mode, out, in, nullptr, batch, 64);
}
int nttmul_pointwise_batch_u32(nttmul_ctx *ctx, uint32_t *c, const uint32_t *a,
                               const uint32_t *b, size_t batch) {
  return run_host(ctx, OP_POINTWISE, c, a, b, batch, 32);
}
int nttmul_pointwise_batch_u64(nttmul_ctx *ctx, uint64_t *c, const uint64_t *a,
                               const uint64_t *b, size_t batch) {
  return run_host(ctx, OP_POINTWISE, c, a, b, batch, 64);
}

static int device_op(nttmul_ctx *ctx, int op, void *c, const void *a, const void *b, size_t batch,
                     int word_bits, int dev, void *stream) {
  const bool two = op == OP_MULTIPLY || op == OP_POINTWISE;
  if (!ctx || (batch && (!c || !a || (two && !b)))) return NTTMUL_EINVAL;
  DevState *d = find_dev(ctx, dev);
  if (!d) return NTTMUL_ENODEV;
  if (const int st = server_quiesce(ctx)) return st;
  DeviceGuard guard;
  HIP_TRY(ctx, hipSetDevice(d->id));
  return run_device(ctx, *d, d->dscr, op, c, a, b, batch, word_bits, (hipStream_t)stream);
}

int nttmul_multiply_batch_device(nttmul_ctx *ctx, void *c, const void *a, const void *b,
                                 size_t batch, int word_bits, int dev, void *stream) {
  return device_op(ctx, OP_MULTIPLY, c, a, b, batch, word_bits, dev, stream);
}
int nttmul_forward_batch_device(nttmul_ctx *ctx, void *out, const void *in, size_t batch,
                                int word_bits, int dev, void *stream) {
  return device_op(ctx, OP_FORWARD, out, in, nullptr, batch, word_bits, dev, stream);
}
int nttmul_inverse_batch_device(nttmul_ctx *ctx, void *out, const void *in, size_t batch,
                                int word_bits, int dev, void *stream) {
  return device_op(ctx, OP_INVERSE, out, in, nullptr, batch, word_bits, dev, stream);
}
int nttmul_transform_device(nttmul_ctx *ctx, unsigned mode, void *out, const void *in,
                            size_t batch, int word_bits, int dev, void *stream) {
  if (mode & ~kXfModes) return NTTMUL_EINVAL;
  return device_op(ctx, OP_XFORM + (int)mode, out, in, nullptr, batch, word_bits, dev, stream);
}
int nttmul_pointwise_batch_device(nttmul_ctx *ctx, void *c, const void *a, const void *b,
                                  size_t batch, int word_bits, int dev, void *stream) {
  return device_op(ctx, OP_POINTWISE, c, a, b, batch, word_bits, dev, stream);
}

int nttmul_fill_random_device(nttmul_ctx *ctx, void *a, void *b, uint64_t p0, size_t count,
                              uint64_t seed, int word_bits, int dev, void *stream) {
  if (!ctx || (count && (!a || !b)) || (word_bits != 32 && word_bits != 64)) return NTTMUL_EINVAL;
  if (word_bits == 32 && ctx->plan.q > 0xFFFFFFFFull) return NTTMUL_EINVAL;
  DevState *d = find_dev(ctx, dev);
  if (!d) return NTTMUL_ENODEV;
  if (const int st = server_quiesce(ctx)) return st;
  DeviceGuard guard;
  HIP_TRY(ctx, hipSetDevice(d->id));
  HIP_TRY(ctx, launch_fill(a, b, ctx->plan.logn, ctx->plan.q, seed, p0, count, word_bits,
                           (hipStream_t)stream));
  return NTTMUL_OK;
}

// ---------------------------------------------------------------------------------------------
// Compat shims: the reference's software-path entry points (n = 256, q = 12289, psi = 1002).
// ---------------------------------------------------------------------------------------------
static nttmul_ctx *g_ctx256[2] = {nullptr, nullptr};  // [0] negacyclic psi, [1] cyclic omega
static std::once_flag g_once256[2];
static std::mutex g_mu256;

static nttmul_ctx *ctx256(int cyclic) {
  std::call_once(g_once256[cyclic], [cyclic] {
    nttmul_params p;
    memset(&p, 0, sizeof(p));
    p.n = 256;
    p.q = 12289;
    // ntt256_tables.h:20-24: psi = 1002, omega = psi^2 = 8595
    p.psi = cyclic ? 8595 : 1002;
    p.flags = cyclic ? NTTMUL_FLAG_CYCLIC : 0;
    p.ndev = 1;
    int st = nttmul_create_ex(&g_ctx256[cyclic], &p);
    if (st) {
      fprintf(stderr, "nttmul: ntt256 context: %s\n", nttmul_strerror(st));
      abort();
    }
  });
  return g_ctx256[cyclic];
}

static void product256(int32_t *c, const int32_t *a, const int32_t *b) {
  nttmul_ctx *ctx = ctx256(0);
  std::lock_guard<std::mutex> lock(g_mu256);
  int st = nttmul_multiply_u32(ctx, (uint32_t *)c, (const uint32_t *)a, (const uint32_t *)b);
  if (st) {
    fprintf(stderr, "nttmul: ntt256 product: %s (%s)\n", nttmul_strerror(st), ctx->err);
    abort();
  }
}

static void transform256(int32_t *a, int cyclic, unsigned mode) {
  nttmul_ctx *ctx = ctx256(cyclic);
  std::lock_guard<std::mutex> lock(g_mu256);
  int st = nttmul_transform_batch_u32(ctx, mode, (uint32_t *)a, (const uint32_t *)a, 1);
  if (st) {
    fprintf(stderr, "nttmul: ntt256 transform: %s (%s)\n", nttmul_strerror(st), ctx->err);
    abort();
  }
}

void ntt256_product1(int32_t *c, int32_t *a, int32_t *b) { product256(c, a, b); }
void ntt256_product4(int32_t *c, int32_t *a, int32_t *b) { product256(c, a, b); }
void ntt_red256_product1(int32_t *c, int32_t *a, int32_t *b) { product256(c, a, b); }
void ntt_red256_product4(int32_t *c, int32_t *a, int32_t *b) { product256(c, a, b); }

// NTT/ntt256.h:20-69 (CT and GS of the same order compute the same transform)
constexpr unsigned kFwdR2S = NTTMUL_XF_FORWARD | NTTMUL_XF_REV2STD;
constexpr unsigned kFwdS2R = NTTMUL_XF_FORWARD | NTTMUL_XF_STD2REV;
constexpr unsigned kInvR2S = NTTMUL_XF_INVERSE | NTTMUL_XF_REV2STD | NTTMUL_XF_UNSCALED;
constexpr unsigned kInvS2R = NTTMUL_XF_INVERSE | NTTMUL_XF_STD2REV | NTTMUL_XF_UNSCALED;
void ntt256_ct_rev2std(int32_t *a) { transform256(a, 1, kFwdR2S); }
void ntt256_gs_rev2std(int32_t *a) { transform256(a, 1, kFwdR2S); }
void ntt256_ct_std2rev(int32_t *a) { transform256(a, 1, kFwdS2R); }
void ntt256_gs_std2rev(int32_t *a) { transform256(a, 1, kFwdS2R); }
void intt256_ct_rev2std(int32_t *a) { transform256(a, 1, kInvR2S); }
void intt256_gs_rev2std(int32_t *a) { transform256(a, 1, kInvR2S); }
void intt256_ct_std2rev(int32_t *a) { transform256(a, 1, kInvS2R); }
void intt256_gs_std2rev(int32_t *a) { transform256(a, 1, kInvS2R); }
void mulntt256_ct_rev2std(int32_t *a) { transform256(a, 0, kFwdR2S); }
void mulntt256_ct_std2rev(int32_t *a) { transform256(a, 0, kFwdS2R); }
void inttmul256_gs_rev2std(int32_t *a) { transform256(a, 0, kInvR2S); }
void inttmul256_gs_std2rev(int32_t *a) { transform256(a, 0, kInvS2R); }

#ifdef NTTMUL_CLOCK_STAMPS
// include/nttmul_diag.h (lib/libnttmul_diag.so only)
int nttmul_diag_clock_stamps(uint64_t *dst, size_t blocks) {
  if (!dst && blocks) return NTTMUL_EINVAL;
  return read_clock_stamps(dst, blocks) == hipSuccess ? NTTMUL_OK : NTTMUL_EHIP;
}
int nttmul_diag_server_stamps(const nttmul_ctx *ctx, uint64_t *dst) {
  if (!ctx || !dst) return NTTMUL_EINVAL;
  if (!ctx->server.box || ctx->last_path != 3) return NTTMUL_EINVAL;
  for (int k = 0; k < 6; k++) dst[k] = __atomic_load_n(&ctx->server.box->stamp[k], __ATOMIC_ACQUIRE);
  dst[6] = ctx->server.host_ns;
  return NTTMUL_OK;
}
#endif

}  // extern "C"
