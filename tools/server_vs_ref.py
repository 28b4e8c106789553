"""One box's per-call comparison for the relinked reference harness (verdict r4 item 5): the
reference's own timing loop (time_testing256.c:175-187, as apps/time_testing_gpu: the same loop
relinked against libnttmul's ntt256_product4, 2,000 calls) against the reference's compiled
ntt256_product4 on one core of the same host (oracle/ref_anchor.c over oracle/_ref), three runs
each, interleaved, in one JSON:
    python tools/server_vs_ref.py > profiles/r5/server_vs_ref_<box>.json
No GPU work in this process: the harness runs as a child program."""
import json
import os
import re
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

APP = os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd", "apps", "time_testing_gpu")
GOLD = os.path.join(ROOT, "tests", "golden")
calls = 2000
gpu, ref = [], []
for _ in range(3):
    out = subprocess.run([APP, os.path.join(GOLD, "coeficientes_a.txt"),
                          os.path.join(GOLD, "coeficientes_b.txt"), str(calls)],
                         capture_output=True, text=True, timeout=120, check=True).stdout
    gpu.append(float(re.search(r"\(([\d.]+) us por chamada", out).group(1)))
    a = O.ref_anchors(reps256=20000, reps1024=10)
    ref.append(a["ntt256_product4 n=256 q=12289"] * 1e6)
model = ""
for line in open("/proc/cpuinfo"):
    if line.startswith("model name"):
        model = line.split(":", 1)[1].strip()
        break
res = {"host": socket.gethostname(), "cpu": model,
       "gpu_shim_us_per_call": gpu, "reference_cpu_us_per_call": ref,
       "gpu_over_cpu_median": sorted(gpu)[1] / sorted(ref)[1],
       "faster": "gpu" if sorted(gpu)[1] < sorted(ref)[1] else "reference cpu",
       "source": "apps/time_testing_gpu (time_testing256.c:175-187 relinked on libnttmul, "
                 f"{calls} calls, device server) vs oracle/ref_anchor.c ntt256_product4 "
                 "(the reference's compiled NTT/ntt256.C, one core), three runs each, interleaved"}
print(json.dumps(res, indent=1))
