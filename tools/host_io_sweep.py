"""PCIe-inclusive rate of the host-buffer ABI path (nttmul_multiply_batch_u32 on host arrays, the
FPGA transaction of NTT_PCIECommunicationv2.c:164-229) at C3, pageable and page-locked, over the
context's copy_threads knob (host threads splitting each staging copy, include/nttmul.h):

    python tools/host_io_sweep.py [--batch 65536] [--threads 4,8,16] [--reps 3] > out.json

Every configuration's result is compared with the first one's (identical products)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd"))
import numpy as np  # noqa: E402
import nttmul  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--q", type=int, default=2013265921)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--threads", default="4,8,16")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    n, q, batch = args.n, args.q, args.batch
    rng = np.random.default_rng(1)
    a = (rng.integers(0, q, size=(batch, n), dtype=np.uint64)).astype(np.uint32)
    b = (rng.integers(0, q, size=(batch, n), dtype=np.uint64)).astype(np.uint32)
    ap_, bp_, cp_ = (nttmul.host_empty(a.shape, np.uint32) for _ in range(3))
    ap_[...] = a
    bp_[...] = b
    out = {"n": n, "q": q, "batch": batch, "bytes_over_pcie": 3 * n * 4 * batch, "runs": []}
    ref = None
    for t in [int(x) for x in args.threads.split(",")]:
        with nttmul.Context(n, q, copy_threads=t) as ctx:
            c = np.empty_like(a)
            ctx.multiply(a[:1], b[:1])                      # staging buffers allocated once
            for kind in ("pageable", "pinned"):
                best = None
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    if kind == "pageable":
                        ctx.multiply(a, b, out=c)
                    else:
                        ctx.multiply(ap_, bp_, out=cp_)
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                res = c if kind == "pageable" else cp_
                if ref is None:
                    ref = res.copy()
                out["runs"].append({"copy_threads": t, "kind": kind, "seconds": best,
                                    "m_polymults_per_s": batch / best / 1e6,
                                    "gb_per_s_over_pcie": out["bytes_over_pcie"] / best / 1e9,
                                    "host_path": ctx.last_host_path(),
                                    "identical": bool(np.array_equal(res, ref))})
                print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
