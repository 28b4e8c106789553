"""C2 per-step host cost: how long the host takes to enqueue one n = 1024 x 4096 product through
(a) the Python wrapper with torch tensors (bench.py's step), (b) the wrapper with integer device
pointers, (c) the C ABI function itself with pre-converted ctypes arguments; and the GPU time per
step (HIP events) for each, rotating over 16 buffer sets.  If the enqueue time per step is at or
above the kernel time the GPU waits for the host."""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd"))
import nttmul  # noqa: E402

n, q, batch, rot, steps = 1024, 2013265921, 4096, 16, 3000
ctx = nttmul.Context(n, q)
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev)
sp = stream.cuda_stream
sets = []
for _ in range(rot):
    a = torch.empty(batch * n, dtype=torch.int32, device=dev)
    b = torch.empty_like(a)
    ctx.fill_random_device(a, b, 0, batch, 32, stream=sp)
    sets.append((a, b, torch.empty_like(a)))
ptrs = [tuple(t.data_ptr() for t in s) for s in sets]
fn = ctx._lib.nttmul_multiply_batch_device
cargs = [(ctx._h, ctypes.c_void_p(c), ctypes.c_void_p(a), ctypes.c_void_p(b), ctypes.c_size_t(batch),
          ctypes.c_int(32), ctypes.c_int(0), ctypes.c_void_p(sp)) for a, b, c in ptrs]


def wrap_tensor(i):
    a, b, c = sets[i % rot]
    ctx.multiply_device(c, a, b, batch, 32, stream=sp)


def wrap_int(i):
    a, b, c = ptrs[i % rot]
    ctx.multiply_device(c, a, b, batch, 32, stream=sp)


def raw(i):
    st = fn(*cargs[i % rot])
    if st:
        raise RuntimeError(st)


out = {}
for name, f in [("wrapper_tensors", wrap_tensor), ("wrapper_ints", wrap_int), ("c_abi", raw)] * 2:
    for i in range(200):
        f(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    t0 = time.perf_counter()
    for i in range(steps):
        f(i)
    t1 = time.perf_counter()
    e1.record(stream)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out.setdefault(name, []).append({"enqueue_us_per_step": (t1 - t0) / steps * 1e6,
                                     "wall_us_per_step": (t2 - t0) / steps * 1e6,
                                     "gpu_us_per_step": e0.elapsed_time(e1) / steps * 1e3})
    print(name, out[name][-1], flush=True)
# host-only cost of the wrapper's argument checks (no launch)
t0 = time.perf_counter()
for i in range(steps):
    a, b, c = sets[i % rot]
    [nttmul._dev_arg(t, batch, n, 32, 0) for t in (c, a, b)]
out["dev_arg_checks_us"] = (time.perf_counter() - t0) / steps * 1e6
print(json.dumps(out))
os.makedirs(os.path.join(ROOT, "gpurun_out", "r3_host"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "r3_host", "c2_host_overhead.json"), "w"), indent=1)
