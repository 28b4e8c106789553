"""Board power of the two kinds of work in a C5 step, separately: an HBM stream at the column
passes' rate (a 1 GiB device copy: read + write, no arithmetic) and the C3 product (VALU-bound,
at the cap), then the C5 product itself.  If the stream draws well under the 1,400 W cap, the
column passes leave power unused that an overlapped design could spend.
    python tools/r3/power_phases.py > out.json"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
import nttmul  # noqa: E402

dev = torch.device("cuda", 0)
props = torch.cuda.get_device_properties(dev)
try:
    bdf = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}"
except AttributeError:
    bdf = ""
reader = bench.power_reader(bdf, 0)
sync = torch.cuda.synchronize
out = {}

# 1. HBM stream: 1 GiB copy per step (2 GiB of traffic), the column passes' access shape
src = torch.empty(1 << 28, dtype=torch.int32, device=dev).fill_(1)
dst = torch.empty_like(src)
copy = lambda: dst.copy_(src)  # noqa: E731
bench.settle(copy, 200, sync)
t0 = time.perf_counter()
for _ in range(50):
    copy()
sync()
dt = (time.perf_counter() - t0) / 50
out["hbm_copy_1GiB"] = {"ms_per_step": dt * 1e3, "tb_per_s": 2 * (1 << 30) / dt / 1e12,
                        "power": bench.power_probe(copy, sync, 4.0, reader)}
del src, dst

# 2. the product kernels: C3 (one launch) and C5 (three launches)
for name, n, q, batch, wb in (("c3", 4096, 2013265921, 65536, 32),
                              ("c5", 65536, 0x3FFFFFFFFFE80001, 1024, 64)):
    ctx = nttmul.Context(n, q, ndev=1, first_dev=0)
    dt_ = torch.int32 if wb == 32 else torch.int64
    a = torch.empty(batch * n, dtype=dt_, device=dev)
    b, c = torch.empty_like(a), torch.empty_like(a)
    s = torch.cuda.current_stream(dev).cuda_stream
    ctx.fill_random_device(a, b, 0, batch, wb, stream=s)
    step = lambda: ctx.multiply_device(c, a, b, batch, wb, stream=s)  # noqa: E731
    bench.settle(step, 200, sync)
    t0 = time.perf_counter()
    for _ in range(50):
        step()
    sync()
    dt = (time.perf_counter() - t0) / 50
    out[name] = {"ms_per_step": dt * 1e3, "power": bench.power_probe(step, sync, 4.0, reader, batch)}
    del a, b, c, ctx
print(json.dumps(out, indent=1))
