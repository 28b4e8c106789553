#!/usr/bin/env python3
"""Benchmark of the MI355X NTT polynomial multiplier (BASELINE.json metric).

One "step" = one batched product c = a * b mod (x^n + 1, q) over this rank's shard of
synthetic polynomials already resident in HBM (generated on the device from the counter-based
splitmix64 stream of SURVEY §8d, so every rank owns a contiguous slice [p0, p0 + batch) of one
global batch and no input crosses PCIe or xGMI).  Scaling is weak: each GPU multiplies
--batch-per-gpu polynomials per step; shards are independent, there is no collective on the data
path and no RCCL at all: torch.distributed runs on gloo over CPU tensors and provides only the
barrier and the max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--settle-ms 200] [--n 4096] [--q 2013265921]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Prints ONE JSON line on rank 0 (fields documented in DESIGN.md §Measurement).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd"))

METRIC = "polymults/sec (n=4096, 32-bit q) at 1/2/4/8 MI355X; % HBM roofline"
# --op: the product (the BASELINE metric) or one of SURVEY §8(f) row 1's standalone steps on
# either side of it, measured the same way: (unit, words moved per polynomial / n)
OPS = {"multiply": ("polymults/s", 3), "forward": ("forward NTTs/s", 2),
       "inverse": ("inverse NTTs/s", 2), "pointwise": ("pointwise products/s", 3)}
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SEED = 0x4E54544D554C


def shard(global_batch: int, rank: int, world: int):
    """Contiguous slice [p0, p1) of the global batch owned by `rank`."""
    p0 = global_batch * rank // world
    p1 = global_batch * (rank + 1) // world
    return p0, p1


def timed_steps(step, steps: int, warmup: int, sync, barrier):
    """W untimed warmup steps, then K timed steps bracketed by barrier + device sync on both
    sides (the driver's contract); returns the wall seconds of the K steps on this rank."""
    for _ in range(warmup):
        step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier()
    sync()
    return time.perf_counter() - t0


def settle(step, ms: float, sync, clock=time.perf_counter):
    """Run the hot path, untimed and before the W warm-up steps, until `ms` of wall time have
    passed, in synchronised chunks that double while a chunk takes under 10 ms (so a fast step is
    never queued far ahead of the device).  On an idle MI355X the first ~40 ms of C3 launches run
    slower than the sustained rate (profiles/r3/warm/ramp.txt: launches 0-4 1.22 ms, 10-19 1.07,
    from 40 ms on 0.986; out.txt: W=0/5 K=20 58.5/61.0 M/s, W=50 K=100 66.7, W=200 K=20 66.4 on
    one box); the driver's --warmup 5 is 5 ms at C3.
    Returns (steps run, wall ms)."""
    if ms <= 0:
        return 0, 0.0
    t0 = clock()
    n, chunk = 0, 1
    while True:
        c0 = clock()
        for _ in range(chunk):
            step()
        sync()
        n += chunk
        if (clock() - t0) * 1e3 >= ms:
            return n, (clock() - t0) * 1e3
        if (clock() - c0) * 1e3 < 10.0:
            chunk *= 2


def max_over_ranks(x: float, dist, device=None) -> float:
    """Max of a per-rank float over the (gloo) process group; identity when not distributed.
    A CPU tensor: the control plane never touches the GPUs or RCCL."""
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_ranks(row, dist):
    """Every rank's row of floats, in rank order (gloo all_gather of a CPU tensor); [row] when
    not distributed."""
    import torch
    t = torch.tensor(row, dtype=torch.float64)
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [list(row)]
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [x.tolist() for x in out]


def rank_summary(rows, steps: int, bytes_per_unit: int, world: int, wall_max: float):
    """Per-rank rates (units per second over each rank's own timed wall time, and over its
    event-timed kernel time) and the aggregate roofline of the whole job: every rank's
    algorithmic bytes over the max-over-ranks wall time, against N x the HBM peak (a slow rank
    shows here, not in rank 0's event-timed roofline.frac)."""
    rates = [cnt * steps / wall for wall, _, cnt in rows]
    kern_rates = [cnt / (kms * 1e-3) for _, kms, cnt in rows]
    total_bytes = sum(cnt for _, _, cnt in rows) * bytes_per_unit * steps
    achieved = total_bytes / wall_max / 1e9
    return ({"achieved": achieved, "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
             "frac": achieved / (HBM_PEAK_GBS * world),
             "source": "all ranks' algorithmic bytes over the max-over-ranks wall time of the K "
                       "timed steps, against N x 8 TB/s"},
            {"rates": rates, "min": min(rates), "max": max(rates),
             "kernel_rates": kern_rates, "kernel_ms": [kms for _, kms, _ in rows],
             "unit": "units/s per rank (own wall time; kernel_rates: own HIP-event kernel time)"})


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--q", type=int, default=2013265921)
    ap.add_argument("--batch-per-gpu", type=int, default=None,
                    help="polymults per GPU per step (default: C3's 65536 per GPU at 1, 2 and 4 "
                         "ranks; at 8 ranks C4's 131072, i.e. BASELINE configs[3]'s 2^20 split "
                         "across 8 GPUs)")
    ap.add_argument("--word-bits", type=int, default=0, help="32/64 coefficient storage (0: auto)")
    ap.add_argument("--op", choices=sorted(OPS), default="multiply",
                    help="multiply (the BASELINE metric); forward / inverse / pointwise time the "
                         "standalone batched entry points (nttmul_forward/inverse/pointwise_batch_"
                         "device, SURVEY 8(f) row 1) with the same contract, not the headline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-io", action="store_true",
                    help="also time the host-buffer ABI path (PCIe-inclusive; never the value)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target wall time of the CPU-baseline sample")
    ap.add_argument("--rotate", type=int, default=0,
                    help="cycle the steps over this many distinct (a, b, c) buffer sets, so a "
                         "batch smaller than the Infinity Cache is still read from HBM "
                         "(0: auto = enough sets for 3 x 256 MiB when the batch fits in it, else 1)")
    ap.add_argument("--streams", type=int, default=1,
                    help="alternate consecutive steps over this many HIP streams (default 1; 2 "
                         "overlaps one launch's tail with the next one's ramp: a C2-sized batch "
                         "is a single generation of workgroups)")
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="before the W warm-up steps, run the hot path untimed for this long so "
                         "the card leaves its idle clock state (reported as 'settle'; 0 disables)")
    ap.add_argument("--power-seconds", type=float, default=4.0,
                    help="after the timed region, keep stepping this long while amd-smi samples "
                         "board power and clocks (rank 0 at N=1; 0 disables)")
    ap.add_argument("--clock-seconds", type=float, default=2.0,
                    help="after the power probe, run the same product from the diagnostic build "
                         "lib/libnttmul_diag.so this long and report the in-kernel clock "
                         "(rank 0 at N=1; 0 disables)")
    ap.add_argument("--dump-samples", default="",
                    help="write <prefix>.rank<r>.npz with sampled products of this rank's slice "
                         "(checked against the oracle by tests/test_gpu_parity.py)")
    return ap.parse_args(argv)


C3_BATCH = 65536             # BASELINE configs[2]: n = 4096, batch 65536 on one GPU
C4_GLOBAL = 1 << 20         # BASELINE configs[3]: n = 4096, batch 2^20 split across 8 GPUs


def default_batch(n: int, world: int) -> int:
    """Polymults per GPU per step when --batch-per-gpu is not given: C3's 65536 on 1, 2 and 4
    GPUs (so per-GPU work is C3's), and at 8 GPUs C4's 2^20 / 8 = 131072, so the driver's 8-GPU
    line is BASELINE's C4 workload (one C3-sized kernel rate either way: the product kernel's
    per-GPU throughput does not depend on the batch beyond a few generations of workgroups)."""
    if n == 4096 and world == 8:
        return C4_GLOBAL // 8
    return C3_BATCH


def cpu_baseline(n: int, q: int, target_s: float):
    """The oracle's psi-merged lazy-Shoup port of the reference's optimized path (oracle/), OpenMP
    over the batch on this host's cores; bounded sample sized to ~target_s seconds.  Beside it
    (BASELINE.md §3): the ports of the unoptimized CT (ntt256.C:5-13) and GS (:16-24) sequences
    at the same (n, q), and the reference's own compiled objects as single-core anchors where
    they can run (n = 256 / 1024, q = 12289; oracle/ref_anchor.c)."""
    import numpy as np
    from oracle import oracle as O

    cores = host_cores()
    threads = cores["threads"]
    P = O.Plan(n, q)
    if q >= (1 << 31):
        return None
    per = max(64, threads * 16)
    a, b = O.fill_inputs(n, q, 0, per)
    a32 = a.astype(np.uint32)
    b32 = b.astype(np.uint32)
    _, t = P.fast_batch_u32(a32, b32, threads)          # warm + calibrate
    reps = max(1, int(target_s / max(t, 1e-6)))
    total_t = 0.0
    for _ in range(reps):
        _, t = P.fast_batch_u32(a32, b32, threads)
        total_t += t
    value = per * reps / total_t
    variants = {}
    for gs, name in ((False, "ct_unoptimized_port"), (True, "gs_unoptimized_port")):
        _, t = P.product_batch(a, b, gs, threads)       # warm + calibrate
        r = max(1, int(0.15 * target_s / max(t, 1e-6)))
        tt = sum(P.product_batch(a, b, gs, threads)[1] for _ in range(r))
        variants[name] = {"value": per * r / tt, "unit": "polymults/s",
                          "us_per_polymult_per_core": tt / (per * r) * threads * 1e6}
    anchors = {k: {"us_per_polymult": v * 1e6, "cores": 1} for k, v in O.ref_anchors().items()}
    c1 = c1_single(target_s=min(2.0, 0.2 * target_s))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": value, "unit": "polymults/s", "cores": threads, "kind": "port",
            "us_per_polymult_per_core": threads / value * 1e6,
            "sample": f"{per * reps} polymults (n={n}, q={q}) = {reps} passes over {per} "
                      f"counter-based inputs, OpenMP {threads} threads ({model}), "
                      f"{total_t:.1f} s, oracle/nttmul_oracle.c orc_fast_batch_u32",
            "host_cores": cores,
            "c1": c1,
            "variants": variants,
            "reference_anchors": anchors or "oracle/_ref not built (no reference tree)"}


def host_cores() -> dict:
    """The host cores this process may use, and the OpenMP thread count the CPU baseline takes:
    every core of the affinity mask, capped by the cgroup CPU quota and by OMP_NUM_THREADS when
    either is set (the GPU box exports OMP_NUM_THREADS = its per-GPU CPU share)."""
    total = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = total
    quota = None
    try:  # cgroup v2: "<quota> <period>" or "max <period>"
        qs, ps = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if qs != "max":
            quota = max(1, int(int(qs) / int(ps)))
    except (OSError, ValueError):
        pass
    omp_env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    threads = min(x for x in (affinity, quota, omp_env) if x)
    limits = [k for k, v in (("affinity", affinity), ("cgroup cpu.max", quota),
                             ("OMP_NUM_THREADS", omp_env)) if v == threads]
    return {"threads": threads, "os_cpu_count": total, "sched_getaffinity": affinity,
            "cgroup_cpu_quota": quota, "OMP_NUM_THREADS": omp_env,
            "rule": f"min(affinity, cgroup quota, OMP_NUM_THREADS) = {threads} "
                    f"(set by {', '.join(limits)})"}


def c1_single(n: int = 1024, q: int = 2013265921, target_s: float = 2.0):
    """BASELINE.json configs[0] (C1): the unoptimized Cooley-Tukey product (ntt256.C:5-13
    sequence, restated at this (n, q)) on ONE host core, ONE polymult per call, timed as
    time_testing256.c:147-187 (inputs restored untimed, CLOCK_MONOTONIC around each call,
    averaged); checked against the oracle's merged product before it is reported."""
    from oracle import oracle as O
    P = O.Plan(n, q)
    a, b = O.fill_inputs(n, q, 0, 1)
    c, t = P.time_single(a[0], b[0], gs=False, reps=30)      # time_testing256.c: 30 calls
    reps = max(30, int(target_s / max(t, 1e-9)))
    c, t = P.time_single(a[0], b[0], gs=False, reps=reps)
    ok = bool((c == P.product_merged(a[0], b[0])).all())
    return {"value": 1.0 / t, "unit": "polymults/s", "us_per_polymult": t * 1e6, "cores": 1,
            "n": n, "q": q, "kind": "port", "matches_oracle": ok,
            "sample": f"{reps} single products (counter-based input 0), ntt256.C:5-13 CT sequence "
                      "(oracle/nttmul_oracle.c orc_time_single), one thread"}


def host_io(ctx, a_dev, b_dev, batch: int, n: int, wb: int, reps: int = 3):
    """PCIe-inclusive rate of the host-buffer ABI path (nttmul_multiply_batch_u*: H2D a, b ->
    product -> D2H c, the FPGA transaction of NTT_PCIECommunicationv2.c:164-229), same inputs."""
    import numpy as np
    dt = np.uint32 if wb == 32 else np.uint64
    a = a_dev.cpu().numpy().view(dt).reshape(batch, n)
    b = b_dev.cpu().numpy().view(dt).reshape(batch, n)
    import nttmul
    ctx.multiply(a[:1], b[:1])                           # staging buffers allocated once

    def best_of(fn):
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            t = time.perf_counter() - t0
            best = t if best is None else min(best, t)
        return best

    res = {"c": np.empty_like(a)}
    res["c"][...] = 0     # the caller's output buffer, allocated and touched once (a fresh array
    #                       per call would add its first-touch page faults: ~65 ms per GiB)
    best = best_of(lambda: ctx.multiply(a, b, out=res["c"]))
    line = {"value": batch / best, "unit": "polymults/s", "seconds": best,
            "bytes_over_pcie": 3 * n * (wb // 8) * batch,
            "note": "pageable host numpy buffers (the output allocated once and reused) through "
                    "nttmul_multiply_batch (PCIe-inclusive, staged by host threads), best of "
                    f"{reps}; reported beside, never the bench value"}
    try:  # the same call on page-locked buffers (nttmul_host_alloc): direct DMA, no staging
        ap, bp = nttmul.host_empty(a.shape, dt), nttmul.host_empty(a.shape, dt)
        cp = nttmul.host_empty(a.shape, dt)
        ap[...] = a
        bp[...] = b
        tp = best_of(lambda: ctx.multiply(ap, bp, out=cp))
        line["pinned"] = {"value": batch / tp, "unit": "polymults/s", "seconds": tp,
                          "matches_pageable": bool(np.array_equal(cp, res["c"])),
                          "note": "a, b, c in nttmul_host_alloc memory: the copy engines DMA "
                                  "the chunks directly (PCIe-bound)"}
    except Exception as e:  # reported beside, never required
        line["pinned"] = {"error": str(e)}
    return line


def _profile_entry(name: str, n: int, q: int, kernels):
    """The entry of profiles/<name> measured on this (n, q) with exactly these kernels:
    `kernels` = {kernel_key: hash} of the kernels one step dispatches (nttmul.dispatched_kernel_
    hashes), compared kernel by kernel with the entry's own "kernels" record.  A profile of any
    other machine code -- or an entry without per-kernel hashes -- is never reported (fails
    closed); edits of other kernels or of host code leave a matching entry valid."""
    if not kernels:
        return None
    try:
        data = json.load(open(os.path.join(ROOT, "profiles", name)))
    except (OSError, ValueError):
        return None
    for e in data.get("entries", []):
        if (e.get("n") == n and e.get("q") == q and e.get("batch")
                and e.get("kernels") == dict(kernels)):
            return e
    return None


def _kernels_tag(kernels) -> str:
    return ", ".join(f"{k} {h}" for k, h in (kernels or {}).items()) or "none"


def load_traffic(n: int, q: int, batch: int, kernels):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of these kernels
    (profiles/pmc_traffic.json, tools/summarize_profile.py), scaled to this batch; with its
    source, or (None, reason)."""
    e = _profile_entry("pmc_traffic.json", n, q, kernels)
    if e is None:
        return None, f"no PMC profile of kernels [{_kernels_tag(kernels)}] at n={n}, q={q}"
    return (e["hbm_bytes_per_launch"] * batch / e["batch"],
            f"profiles/pmc_traffic.json <- {e['source']} (kernels {_kernels_tag(kernels)}; "
            f"batch {e['batch']}, {e['method']})")


def load_valu_bound(n: int, q: int, kernels):
    """VALU issue cycles of one step's kernels, from their ISA listings (profiles/valu_bound.json,
    tools/valu_bound.py), or None."""
    return _profile_entry("valu_bound.json", n, q, kernels)


def valu_roofline(vb: dict, count: int, kern_ms: float, source_kernels) -> dict:
    """The bound that binds the product kernels: every dispatched kernel's ISA
    listing priced at the measured issue costs (cycles per wave x waves per polynomial, summed
    over the step's launches), for `count` polynomials over the 1,024 SIMDs at the 2.4 GHz
    maximum clock; implied_clock_ghz = the clock at which the step would run exactly at it."""
    per = []
    total_cycles = 0.0
    for k in vb["per_kernel"]:
        w = k["waves_per_unit"] * count / SIMDS
        total_cycles += k["cycles_per_wave"] * w
        per.append({"kernel": k["kernel"], "valu_per_wave": k["valu_per_wave"],
                    "cycles_per_wave": k["cycles_per_wave"], "waves_per_simd": w,
                    "bound_ms": k["cycles_per_wave"] * w / (MAX_CLOCK_GHZ * 1e9) * 1e3})
    bound_ms = total_cycles / (MAX_CLOCK_GHZ * 1e9) * 1e3
    out = {"bound": "valu", "clock_ghz": MAX_CLOCK_GHZ, "bound_ms": bound_ms,
           "frac": bound_ms / kern_ms, "cycles_per_simd": total_cycles,
           "implied_clock_ghz": total_cycles / (kern_ms * 1e6), "kernels": per,
           "source": f"profiles/valu_bound.json (kernels {_kernels_tag(source_kernels)}): each "
                     "kernel's ISA listing priced at measured issue costs, summed over the step's "
                     "launches, at the 2.4 GHz max clock; implied_clock_ghz = the clock at which "
                     "the step would run exactly at that issue bound"}
    if len(per) == 1:  # single-launch products: the per-wave figures at the top level as before
        out.update(cycles_per_wave=per[0]["cycles_per_wave"],
                   valu_per_wave=per[0]["valu_per_wave"], waves_per_simd=per[0]["waves_per_simd"])
    return out


def code_object_or_none():
    import nttmul
    try:
        return nttmul.code_object_id()
    except (OSError, ValueError):
        return None


def kernels_or_none(names: str):
    """{kernel_key: hash} of the kernels a step dispatches (nttmul_kernel_name string), or None."""
    import nttmul
    try:
        return nttmul.dispatched_kernel_hashes(names)
    except (OSError, ValueError, KeyError):
        return None


def workload_name(n: int, q: int, global_batch: int, world: int) -> str:
    """BASELINE.json config this run matches, else 'custom'."""
    if n == 4096 and q < (1 << 32):
        if world == 8 and global_batch == 1 << 20:
            return "C4"
        if global_batch == 65536 * world:
            return "C3"
    if n == 1024 and global_batch == 4096 * world:
        return "C2"
    if n == 65536 and q >= (1 << 32) and global_batch == 1024 * world:
        return "C5"
    return "custom"


IC_BYTES = 256 << 20        # MI355X Infinity Cache (MI355X_MICROARCH.md)


def buffer_sets(step_bytes: int, requested: int = 0) -> int:
    """Distinct (a, b, c) sets the timed steps cycle over: `requested` if given, else enough
    that a step's working set that fits the Infinity Cache is evicted before it is read again
    (3 x 256 MiB worth of sets), else 1."""
    if requested > 0:
        return requested
    return -(-3 * IC_BYTES // step_bytes) if step_bytes <= IC_BYTES else 1


def _num(x):
    return x if isinstance(x, (int, float)) and not isinstance(x, bool) else None


def power_reader(bdf: str, devno: int):
    """(read, cap_w, index) over the amdsmi library in this process -- read-only queries through
    the kernel driver, no child process -- or None when amdsmi is unavailable.  read() returns one
    sample: socket power (W), shader clock (MHz), gfx activity (%), PPT (package power) limiter
    state.  The GPU is matched by PCI address, else by index."""
    try:
        import amdsmi as S
        S.amdsmi_init()
        hs = S.amdsmi_get_processor_handles()
    except Exception:  # no library, no driver access
        return None
    h, idx = None, None
    for i, x in enumerate(hs):
        try:
            if bdf and str(S.amdsmi_get_gpu_device_bdf(x)).lower().startswith(bdf.lower()):
                h, idx = x, i
        except Exception:
            continue
    if h is None and devno < len(hs):
        h, idx = hs[devno], devno
    if h is None:
        return None
    cap = None
    try:
        c = _num(S.amdsmi_get_power_cap_info(h).get("power_cap"))
        cap = c / 1e6 if c and c > 1e5 else c          # the library reports microwatts
    except Exception:
        pass

    def read():
        row = {}
        try:
            p = S.amdsmi_get_power_info(h)
            row["w"] = next((_num(p.get(k)) for k in ("current_socket_power", "socket_power",
                                                      "average_socket_power")
                             if _num(p.get(k))), None)
        except Exception:
            row["w"] = None
        try:
            row["mhz"] = _num(S.amdsmi_get_clock_info(h, S.AmdSmiClkType.GFX).get("clk"))
        except Exception:
            row["mhz"] = None
        try:
            row["busy"] = _num(S.amdsmi_get_gpu_activity(h).get("gfx_activity"))
        except Exception:
            row["busy"] = None
        try:
            v = S.amdsmi_get_violation_status(h)
            a = v.get("active_ppt_pwr")
            row["ppt"] = a if isinstance(a, bool) else None
            row["ppt_pct"] = _num(v.get("per_ppt_pwr"))
        except Exception:
            row["ppt"], row["ppt_pct"] = None, None
        return row

    return read, cap, idx


def power_probe(step, sync, seconds: float, reader, units_per_step: int = 0):
    """Board power while the timed workload keeps running (the product kernels are
    bound by the package power cap).  After the timed region, extra steps run for `seconds` while
    a thread samples `reader` (power_reader) every 0.2 s; reports the median socket power, the cap,
    the median shader clock and how many busy samples had the PPT limiter engaged."""
    import statistics
    import threading
    if reader is None:
        return None
    read, cap, idx = reader
    done = threading.Event()
    rows = []

    def sample():
        while not done.wait(0.2):
            rows.append(read())

    th = threading.Thread(target=sample, daemon=True)
    t0 = time.perf_counter()
    t_end = t0 + seconds
    nsteps = 0
    th.start()
    while time.perf_counter() < t_end:
        for _ in range(32):
            step()
        sync()
        nsteps += 32
    elapsed = time.perf_counter() - t0
    done.set()
    th.join(timeout=30)
    busy = [r for r in rows if (r.get("busy") or 0) >= 90 and r.get("w")]
    out = {"socket_power_cap_w": cap, "samples": len(rows), "busy_samples": len(busy),
           "amd_smi_gpu": idx,
           "source": f"amdsmi library (in process) sampled every 0.2 s during {seconds:g} s of "
                     "further steps after the timed region; medians over gfx-busy samples"}
    if busy:
        out["socket_power_w_median"] = statistics.median(r["w"] for r in busy)
        if units_per_step:  # board energy per unit of work at the rate of these extra steps
            rate = units_per_step * nsteps / elapsed
            out["rate_during_probe"] = rate
            out["board_uj_per_unit"] = out["socket_power_w_median"] / rate * 1e6
        clk = [r["mhz"] for r in busy if r.get("mhz")]
        if clk:
            out["gfx_clock_mhz_median"] = statistics.median(clk)
        ppt = [r["ppt"] for r in busy if r.get("ppt") is not None]
        if ppt:
            out["ppt_limiter_active"] = f"{sum(ppt)}/{len(ppt)}"
        pct = [r["ppt_pct"] for r in busy if r.get("ppt_pct") is not None]
        if pct:
            out["ppt_violation_pct_median"] = statistics.median(pct)
    return out


def diag_clock(n: int, q: int, wb: int, count: int, a, b, c, devno: int, stream_ptr: int,
               sync, seconds: float = 2.0):
    """The shader clock the product kernel holds, read inside the kernel (MI355X_MICROARCH.md
    'DVFS give-back' item 6): the same product runs from lib/libnttmul_diag.so -- the production
    kernels plus s_memtime / s_memrealtime stamps by thread 0 of each k_rows workgroup
    (include/nttmul_diag.h) -- back to back for `seconds` on the bench's device-resident inputs,
    then the last launch's per-workgroup clocks d(memtime) / d(realtime) x 100 MHz are summarised
    (median over workgroups).  None when the diagnostic library is not built."""
    import ctypes
    import statistics
    import time as _t
    import numpy as np
    import nttmul
    try:
        lib = nttmul.load_diag_library()
    except ImportError:
        return None
    ctx = nttmul.Context(n, q, ndev=1, first_dev=devno, _lib=lib)
    try:
        t0 = _t.perf_counter()
        launches = 0
        while _t.perf_counter() - t0 < seconds:
            for _ in range(16):
                ctx.multiply_device(c, a, b, count, wb, stream=stream_ptr)
            sync()
            launches += 16
        # k_rows workgroups of that launch (products per workgroup: 256 / (n / 16) threads,
        # one 64-thread workgroup per product at n = 1024; n > 4096: 2^(logn - 12) rows each)
        logn = n.bit_length() - 1
        units = count << max(0, logn - 12)
        per_wg = 1 if logn >= 10 else 256 // (n // 16)
        wgs = min(-(-units // per_wg), 1 << 16)
        st = np.zeros(wgs * 4, dtype=np.uint64)
        if lib.nttmul_diag_clock_stamps(st.ctypes.data, wgs) != 0:
            return {"error": "nttmul_diag_clock_stamps failed"}
        st = st.reshape(wgs, 4).astype(np.float64)
        dr = st[:, 3] - st[:, 1]
        ok = dr > 0
        mhz = ((st[ok, 2] - st[ok, 0]) / dr[ok] * 100.0).tolist()
        if not mhz:
            return {"error": "no stamps"}
        mhz.sort()
        return {"clock_ghz_median": statistics.median(mhz) / 1e3,
                "clock_ghz_p10": mhz[len(mhz) // 10] / 1e3, "clock_ghz_p90": mhz[len(mhz) * 9 // 10] / 1e3,
                "workgroups": len(mhz), "launches_before": launches,
                "kernel": ctx.last_kernel_name(),
                "source": "lib/libnttmul_diag.so (production kernels + clock stamps), "
                          f"{launches} launches back to back on the bench inputs, then the last "
                          "launch's per-workgroup d(s_memtime) / d(s_memrealtime) x 100 MHz"}
    finally:
        ctx.close()


MAX_CLOCK_GHZ = 2.4         # MI355X max engine clock (MI355X_MICROARCH.md)
SIMDS = 1024                # 256 CUs x 4 SIMDs


def main(argv=None):
    args = parse(argv)
    import torch
    import torch.distributed as dist
    import nttmul

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    if world > 1:  # control plane only (barrier, max of a float): gloo on CPU tensors, no RCCL
        dist.init_process_group("gloo")
    # one rank per GPU; more ranks than GPUs (the 2-rank rehearsal on a 1-GPU box) share them
    ndev = torch.cuda.device_count()
    devno = local % max(ndev, 1)
    torch.cuda.set_device(devno)
    dev = torch.device("cuda", devno)

    n, q = args.n, args.q
    wb = args.word_bits or (32 if q < (1 << 32) else 64)
    # per-GPU batch: --batch-per-gpu, else default_batch(world) -- C3's 65536 per
    # GPU up to 4 ranks, C4's 2^20 / 8 at 8
    batch = args.batch_per_gpu or default_batch(n, world)
    global_batch = batch * world
    p0, p1 = shard(global_batch, rank, world)
    count = p1 - p0
    wbytes = wb // 8
    unit, words = OPS[args.op]
    alg_bytes = words * n * wbytes * count                # read a (and b) + write the result
    rotate = buffer_sets(alg_bytes, args.rotate)
    nstreams = max(1, args.streams)
    if nstreams > 1:  # each buffer set always goes to the same stream (no cross-stream reuse)
        rotate = -(-max(rotate, nstreams) // nstreams) * nstreams

    ctx = nttmul.Context(n, q, ndev=1, first_dev=devno)
    dt = torch.int32 if wb == 32 else torch.int64
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    # --streams S: consecutive steps alternate over S streams, so one launch's store tail and the
    # next one's load ramp overlap (a batch that is a single generation of workgroups, C2)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(nstreams - 1)]
    sets = []
    for _ in range(rotate):   # identical inputs in every set (same counter range)
        a = torch.empty(count * n, dtype=dt, device=dev)
        b = torch.empty_like(a)
        ctx.fill_random_device(a, b, p0, count, wb, seed=SEED, stream=sptr)
        sets.append((a, b, torch.empty_like(a)))
    state = {"i": 0}

    def step():
        a, b, c = sets[state["i"] % rotate]
        st = streams[state["i"] % nstreams]
        state["i"] += 1
        if args.op == "multiply":
            ctx.multiply_device(c, a, b, count, wb, stream=st.cuda_stream)
        elif args.op == "forward":
            ctx.forward_device(c, a, count, wb, stream=st.cuda_stream)
        elif args.op == "inverse":
            ctx.inverse_device(c, a, count, wb, stream=st.cuda_stream)
        else:
            ctx.pointwise_device(c, a, b, count, wb, stream=st.cuda_stream)

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    events = {"n": 0}

    def timed_step():  # HIP events on the launch stream around the K timed steps
        if events["n"] == args.warmup:
            ev0.record(stream)
            for st in streams[1:]:  # the other streams' timed steps start after ev0
                st.wait_event(ev0)
        step()
        events["n"] += 1
        if events["n"] == args.warmup + args.steps:
            for st in streams[1:]:  # ev1 after every stream's last timed step
                stream.wait_event(st.record_event())
            ev1.record(stream)

    settle_steps, settle_ms = settle(step, args.settle_ms, lambda: torch.cuda.synchronize(dev))
    wall = timed_steps(timed_step, args.steps, args.warmup, lambda: torch.cuda.synchronize(dev),
                       (lambda: dist.barrier()) if world > 1 else (lambda: None))
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    wall_max = max_over_ranks(wall, dist if world > 1 else None)
    rank_rows = gather_ranks([wall, kern_ms, float(count)], dist if world > 1 else None)

    if args.dump_samples:  # sampled products of this rank's slice, at their global positions
        import numpy as np
        a, b, c = sets[(state["i"] - 1) % rotate]
        idx = sorted({0, 1, count // 2, count - 1})
        host = c.view(count, n)[torch.tensor(idx, device=c.device)].cpu().numpy()
        rows = host.view(np.uint32 if wb == 32 else np.uint64).astype(np.uint64)
        np.savez(f"{args.dump_samples}.rank{rank}.npz", p0=p0, p1=p1, idx=np.array(idx),
                 c=rows, n=n, q=q, world=world, global_batch=global_batch)

    if world > 1:
        # every rank's GPU work is done: rank 0 alone goes on to the CPU baseline (the others
        # leave), so its sample runs on a quiet host at every N
        dist.barrier()
    if rank == 0:
        value = global_batch * args.steps / wall_max
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9     # GB/s
        product = args.op == "multiply"
        co = code_object_or_none()
        kname = ((ctx.last_kernel_name() or ctx.kernel_name(wb, count)) if product
                 else f"nttmul_{args.op}_batch_device")
        kernels = kernels_or_none(kname) if product else None
        traffic, traffic_source = (load_traffic(n, q, count, kernels) if kernels and nstreams == 1 else
                                   (None, "PMC profiles are of the product" if not product else
                                    "not attributable: with launches overlapping on several "
                                    "streams each dispatch's counter window holds the others' "
                                    "traffic too (2.01 x at C2, profiles/r6/c2s_pmc.json)"
                                    if nstreams > 1 else f"no per-kernel hashes for {kname}"))
        resident = alg_bytes * rotate <= IC_BYTES
        line = {
            "metric": METRIC if product else
                      f"{unit[:-2]}/sec (n={n}, {'32' if wb == 32 else '64'}-bit words), standalone "
                      "batched entry point (SURVEY 8(f) row 1; not the headline); % HBM roofline",
            "value": value,
            "unit": unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"steps": settle_steps, "ms": round(settle_ms, 1),
                       "note": "untimed hot-path steps before the W warm-up steps, so the card "
                               "is past its idle clock ramp (DESIGN.md §5 'Settle phase')"},
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32" if wb == 32 else "u64",
            "data": "synthetic: splitmix64 counter-based coefficients mod q, generated on device "
                    "(SURVEY §8d, seed 0x4E54544D554C)",
            "config": {"workload": (f"{workload_name(n, q, global_batch, world)}: " if product else
                                    f"{args.op} on {workload_name(n, q, global_batch, world)}'s shape: ") +
                                   f"n={n}, q={q}, batch {batch} polynomials per GPU "
                                   f"(global {global_batch}), device-resident",
                       "op": args.op,
                       "n": n, "q": q, "batch_per_gpu": batch, "global_batch": global_batch,
                       "parallelism": f"batch shards x{world}, no collective",
                       "batch_rule": ("--batch-per-gpu" if args.batch_per_gpu else
                                      "default: 65536 per GPU at 1/2/4 GPUs (C3 per GPU), "
                                      "131072 at 8 (C4 = 2^20 across 8)")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_source,
                         "kernel": kname,
                         "kernel_ms": kern_ms,
                         "alg_bytes_per_launch": alg_bytes,
                         "buffer_sets": rotate,
                         "streams": nstreams,
                         "cache_resident": resident},
            "build": {"code_object": co, "kernels": kernels,
                      "note": "kernels: {kernel: sha256 of its machine code + descriptor} of the "
                              "kernels one step dispatches (nttmul.kernel_hashes); the committed "
                              "profiles below are looked up by these, kernel by kernel"},
            "cpu_baseline": None,
        }
        agg, per_rank = rank_summary(rank_rows, args.steps, words * n * wbytes, world, wall_max)
        line["roofline"]["aggregate"] = agg
        line["ranks"] = per_rank
        if nstreams > 1:
            line["roofline"]["streams_note"] = (
                f"consecutive steps alternate over {nstreams} HIP streams; kernel_ms is the time "
                "per step over the K timed steps (launches overlap, so a single dispatch in a "
                "profiler trace lasts longer)")
        if rotate > 1:
            line["roofline"]["note"] = (
                f"one step's a, b, c ({alg_bytes / 2**20:.0f} MiB) fit the 256 MiB Infinity "
                f"Cache; the steps cycle over {rotate} buffer sets ({rotate * alg_bytes / 2**20:.0f}"
                " MiB) so inputs come from HBM as in a batch that does not fit")
        vb = load_valu_bound(n, q, kernels) if kernels else None
        if vb:  # the bound that binds: integer VALU issue, from this build's ISA
            line["valu_roofline"] = valu_roofline(vb, count, kern_ms, kernels)
        if world == 1 and args.power_seconds > 0:
            try:
                props = torch.cuda.get_device_properties(dev)
                bdf = (f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:"
                       f"{props.pci_device_id:02x}")
            except AttributeError:
                bdf = ""
            try:
                line["power"] = power_probe(step, lambda: torch.cuda.synchronize(dev),
                                            args.power_seconds, power_reader(bdf, devno),
                                            units_per_step=count)
            except Exception as e:  # reported evidence, never required
                line["power"] = {"error": str(e)}
        if world == 1 and args.clock_seconds > 0 and product:
            a, b, c = sets[0]
            try:
                clk = diag_clock(n, q, wb, count, a, b, c, devno, sptr,
                                 lambda: torch.cuda.synchronize(dev), args.clock_seconds)
            except Exception as e:  # reported evidence, never required
                clk = {"error": str(e)}
            if clk:
                line["in_kernel_clock"] = clk
                vr = line.get("valu_roofline")
                if vr and clk.get("clock_ghz_median"):  # the issue bound at the clock actually held
                    g = clk["clock_ghz_median"]
                    vr["in_kernel_clock_ghz"] = g
                    vr["bound_ms_at_in_kernel_clock"] = vr["cycles_per_simd"] / (g * 1e9) * 1e3
                    vr["frac_at_in_kernel_clock"] = vr["bound_ms_at_in_kernel_clock"] / kern_ms
                    if len(vr["kernels"]) > 1:
                        vr["in_kernel_clock_note"] = (
                            "the clock stamps are taken in the row pass (k_rows) only; the bound "
                            "at that clock prices every launch of the step at it")
        if args.host_io and product:
            a, b, _ = sets[0]
            line["host_io"] = host_io(ctx, a, b, count, n, wb)
        if not args.no_cpu_baseline and product:
            try:  # rank 0 only, after every rank's GPU work (the final barrier above)
                line["cpu_baseline"] = cpu_baseline(n, q, args.cpu_seconds)
                if line["cpu_baseline"] and world > 1:
                    line["cpu_baseline"]["note"] = (
                        f"rank 0 of {world}, after the final barrier: the other ranks have left, "
                        "so the sample has the host to itself")
            except Exception as e:  # the baseline is reported, never required
                line["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
