"""Per-launch C3 kernel time from a cold start (HIP events around every launch on the launch
stream): how long the card takes to reach its sustained rate, the reason for bench.py's settle
phase.  python tools/r3/ramp_trace.py [launches] > out.txt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd"))
import torch  # noqa: E402
import nttmul  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
n, q, batch = 4096, 2013265921, 65536
ctx = nttmul.Context(n, q, ndev=1, first_dev=0)
a = torch.empty(batch * n, dtype=torch.int32, device="cuda:0")
b, c = torch.empty_like(a), torch.empty_like(a)
s = torch.cuda.current_stream()
ctx.fill_random_device(a, b, 0, batch, 32, stream=s.cuda_stream)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(N + 1)]
ev[0].record(s)
for i in range(N):
    ctx.multiply_device(c, a, b, batch, 32, stream=s.cuda_stream)
    ev[i + 1].record(s)
torch.cuda.synchronize()
t, acc = [], 0.0
for i in range(N):
    t.append(ev[i].elapsed_time(ev[i + 1]))
for lo, hi in [(0, 5), (5, 10), (10, 20), (20, 40), (40, 60), (60, 100), (100, 200), (200, N)]:
    if lo >= N:
        break
    seg = t[lo:min(hi, N)]
    acc = sum(t[:lo])
    print(f"launches {lo:4d}-{min(hi, N) - 1:4d} (from {acc:7.1f} ms): mean {sum(seg) / len(seg):.4f} ms"
          f"  min {min(seg):.4f}  max {max(seg):.4f}")
