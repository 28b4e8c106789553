#!/usr/bin/env python3
"""Benchmark of the MI355X NTT polynomial multiplier (BASELINE.json metric).

One "step" = one batched product c = a * b mod (x^n + 1, q) over this rank's shard of
synthetic polynomials already resident in HBM (generated on the device from the counter-based
splitmix64 stream of SURVEY §8d, so every rank owns a contiguous slice [p0, p0 + batch) of one
global batch and no input crosses PCIe or xGMI).  Scaling is weak: each GPU multiplies
--batch-per-gpu polynomials per step; shards are independent, there is no collective on the data
path (torch.distributed only provides the barrier and the max-over-ranks time).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 4096] [--q 2013265921]
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


def max_over_ranks(x: float, dist, device) -> float:
    """Max of a per-rank float over the process group (identity when not distributed)."""
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--q", type=int, default=2013265921)
    ap.add_argument("--batch-per-gpu", type=int, default=0,
                    help="0: 65536 (C3) per GPU, or 2^20 / 8 at 8 ranks (C4: batch 2^20 over 8 GPUs)")
    ap.add_argument("--word-bits", type=int, default=0, help="32/64 coefficient storage (0: auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-io", action="store_true",
                    help="also time the host-buffer ABI path (PCIe-inclusive; never the value)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target wall time of the CPU-baseline sample")
    return ap.parse_args(argv)


def cpu_baseline(n: int, q: int, target_s: float):
    """The oracle's psi-merged lazy-Shoup port of the reference's optimized path (oracle/), OpenMP
    over the batch on this host's cores; bounded sample sized to ~target_s seconds.  Beside it
    (BASELINE.md §3): the ports of the unoptimized CT (ntt256.C:5-13) and GS (:16-24) sequences
    at the same (n, q), and the reference's own compiled objects as single-core anchors where
    they can run (n = 256 / 1024, q = 12289; oracle/ref_anchor.c)."""
    import numpy as np
    from oracle import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or O.num_threads()
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
                      f"counter-based inputs, OpenMP {threads} threads of {os.cpu_count()} "
                      f"({model}), {total_t:.1f} s, oracle/nttmul_oracle.c orc_fast_batch_u32",
            "variants": variants,
            "reference_anchors": anchors or "oracle/_ref not built (no reference tree)"}


def host_io(ctx, a_dev, b_dev, batch: int, n: int, wb: int, reps: int = 3):
    """PCIe-inclusive rate of the host-buffer ABI path (nttmul_multiply_batch_u*: H2D a, b ->
    product -> D2H c, the FPGA transaction of NTT_PCIECommunicationv2.c:164-229), same inputs."""
    import numpy as np
    dt = np.uint32 if wb == 32 else np.uint64
    a = a_dev.cpu().numpy().view(dt).reshape(batch, n)
    b = b_dev.cpu().numpy().view(dt).reshape(batch, n)
    ctx.multiply(a[:1], b[:1])                           # staging buffers allocated once
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.multiply(a, b)
        t = time.perf_counter() - t0
        best = t if best is None else min(best, t)
    return {"value": batch / best, "unit": "polymults/s", "seconds": best,
            "bytes_over_pcie": 3 * n * (wb // 8) * batch,
            "note": "host numpy buffers through nttmul_multiply_batch (PCIe-inclusive), best of "
                    f"{reps}; reported beside, never the bench value"}


def load_traffic(n: int, q: int, batch: int):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), if one matches."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        data = json.load(open(path))
    except (OSError, ValueError):
        return None
    for e in data.get("entries", []):   # per-polymult bytes of a measured batch, scaled
        if e.get("n") == n and e.get("q") == q and e.get("batch"):
            return e["hbm_bytes_per_launch"] * batch / e["batch"]
    return None


def load_valu_bound(n: int, q: int, batch: int):
    """VALU-issue bound of the product kernel (profiles/r1_valu_bound.json, tools/valu_bound.py):
    cycles per wave from the ISA x waves per SIMD / the clock the kernel sustains (PMC)."""
    path = os.path.join(ROOT, "profiles", "r1_valu_bound.json")
    try:
        data = json.load(open(path))
    except (OSError, ValueError):
        return None
    for e in data.get("entries", []):   # waves per SIMD scale with the batch
        if e.get("n") == n and e.get("q") == q and e.get("batch"):
            return dict(e, valu_bound_ms=e["valu_bound_ms"] * batch / e["batch"])
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


def arith_name(q: int) -> str:
    """Kernel arithmetic class the library dispatches to for q (modarith.hpp)."""
    if q < (1 << 30):
        return "Arith32H"
    if q < (1 << 31):
        return "Arith32"
    return "Arith32W" if q < (1 << 32) else "Arith64"


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
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    n, q = args.n, args.q
    wb = args.word_bits or (32 if q < (1 << 32) else 64)
    # weak scaling: C3's 65536 polymults per GPU; at 8 ranks the global batch is C4's 2^20
    batch = args.batch_per_gpu or ((1 << 20) // world if world == 8 else 65536)
    global_batch = batch * world
    p0, p1 = shard(global_batch, rank, world)

    ctx = nttmul.Context(n, q, ndev=1, first_dev=local)
    dt = torch.int32 if wb == 32 else torch.int64
    a = torch.empty((p1 - p0) * n, dtype=dt, device=dev)
    b = torch.empty_like(a)
    c = torch.empty_like(a)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    ctx.fill_random_device(a, b, p0, p1 - p0, wb, seed=SEED, stream=sptr)

    def step():
        ctx.multiply_device(c, a, b, p1 - p0, wb, stream=sptr)

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    events = {"n": 0}

    def timed_step():  # HIP events on the launch stream around the K timed steps
        if events["n"] == args.warmup:
            ev0.record(stream)
        step()
        events["n"] += 1
        if events["n"] == args.warmup + args.steps:
            ev1.record(stream)

    wall = timed_steps(timed_step, args.steps, args.warmup, lambda: torch.cuda.synchronize(dev),
                       (lambda: dist.barrier()) if world > 1 else (lambda: None))
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    wall_max = max_over_ranks(wall, dist if world > 1 else None, dev)

    if rank == 0:
        value = global_batch * args.steps / wall_max
        wbytes = wb // 8
        alg_bytes = 3 * n * wbytes * (p1 - p0)           # read a, b + write c, per launch
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9     # GB/s
        single_launch = n <= 4096
        traffic = load_traffic(n, q, batch)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "polymults/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32" if wb == 32 else "u64",
            "data": "synthetic: splitmix64 counter-based coefficients mod q, generated on device "
                    "(SURVEY §8d, seed 0x4E54544D554C)",
            "config": {"workload": f"{workload_name(n, q, global_batch, world)}: "
                                   f"n={n}, q={q}, batch {batch} polymults per GPU "
                                   f"(global {global_batch}), device-resident",
                       "n": n, "q": q, "batch_per_gpu": batch, "global_batch": global_batch,
                       "parallelism": f"batch shards x{world}, no collective"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": (f"k_rows<{arith_name(q)},u32,u32,{n.bit_length() - 1},0>"
                                    if (single_launch and wb == 32)
                                    else "polymul (all launches of one step)"),
                         "kernel_ms": kern_ms,
                         "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": None,
        }
        vb = load_valu_bound(n, q, batch) if single_launch and wb == 32 else None
        if vb:  # the bound that binds: integer VALU issue at the sustained clock
            line["valu_roofline"] = {"bound": "valu", "cycles_per_wave": vb["cycles_per_wave"],
                                     "valu_per_wave": vb["valu_per_wave"],
                                     "clock_ghz": vb["clock_ghz"], "bound_ms": vb["valu_bound_ms"],
                                     "frac": vb["valu_bound_ms"] / kern_ms}
        if args.host_io:
            line["host_io"] = host_io(ctx, a, b, p1 - p0, n, wb)
        if world == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(n, q, args.cpu_seconds)
            except Exception as e:  # the baseline is reported, never required
                line["cpu_baseline"] = {"error": str(e)}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
