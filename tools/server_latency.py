"""Per-call latency of a single small host product (n = 256, q = 12289: the reference's
ntt256_product4 shape) through the resident device server vs a kernel launch per call, and the
server's own timeline from lib/libnttmul_diag.so (nttmul_diag_server_stamps): request seen ->
a, b loaded -> product computed -> c stored and released, plus the host's go -> done-seen time.
    python tools/server_latency.py [--calls 2000] > out.json"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd"))
import numpy as np  # noqa: E402
import nttmul  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--calls", type=int, default=2000)
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--q", type=int, default=12289)
ap.add_argument("--batch", type=int, default=1, help="products per call (n x batch <= 1024)")
args = ap.parse_args()
rng = np.random.default_rng(7)
shape = args.n if args.batch == 1 else (args.batch, args.n)
a = rng.integers(0, args.q, shape, dtype=np.uint32)
b = rng.integers(0, args.q, shape, dtype=np.uint32)
res = {"n": args.n, "q": args.q, "batch": args.batch, "calls": args.calls}
outs = {}


def timed(ctx, calls):
    c = np.empty(shape, np.uint32)
    ctx.multiply(a, b, out=c)
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter_ns()
        ctx.multiply(a, b, out=c)
        ts.append((time.perf_counter_ns() - t0) / 1e3)
    ts.sort()
    return {"us_p50": ts[len(ts) // 2], "us_p10": ts[len(ts) // 10], "us_p90": ts[len(ts) * 9 // 10],
            "us_mean": statistics.mean(ts), "path": ctx._lib.nttmul_last_host_path(ctx._h)}, c


for name, lib, srv in (("server", None, 0), ("launch_per_call", None, -1),
                       ("server_diag", "diag", 0)):
    L = nttmul.load_diag_library() if lib == "diag" else None
    with nttmul.Context(args.n, args.q, small_server=srv, _lib=L) as ctx:
        row, c = timed(ctx, args.calls)
        if name == "server_diag":
            L.nttmul_diag_server_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            st = np.zeros(7, np.uint64)
            seen = []
            for _ in range(200):
                ctx.multiply(a, b, out=c)
                if L.nttmul_diag_server_stamps(ctx._h, st.ctypes.data) == 0:
                    s = st.astype(np.int64)
                    seen.append([(s[1] - s[0]) * 10.0, (s[2] - s[1]) * 10.0, (s[3] - s[2]) * 10.0,
                                 (s[3] - s[0]) * 10.0, float(s[6]),
                                 (s[5] - s[4]) / max(1, (s[2] - s[1])) * 100.0])
            if seen:
                cols = list(zip(*seen))
                keys = ["load_ns", "compute_ns", "store_release_ns", "gpu_busy_ns", "host_go_to_done_ns",
                        "compute_clock_mhz"]
                row["timeline_median"] = {k: statistics.median(v) for k, v in zip(keys, cols)}
                row["timeline_median"]["host_minus_gpu_ns"] = (row["timeline_median"]["host_go_to_done_ns"]
                                                              - row["timeline_median"]["gpu_busy_ns"])
        res[name] = row
        outs[name] = c.copy()
res["outputs_identical"] = all(np.array_equal(outs["launch_per_call"], v) for v in outs.values())
print(json.dumps(res, indent=1))
