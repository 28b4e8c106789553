"""Board energy per VALU lane-op of each instruction kind in tools/r4/valu_energy.hip (DESIGN §4,
verdict r3 item 3).  Every kind runs back to back for --seconds while bench.power_probe samples
socket power through amdsmi (in process); the lane-op rate comes from wall time over the same
launches and the clock from the kernel's own s_memtime / s_memrealtime stamps (median over
workgroups of the last launch).  pJ per lane-op = median power / lane-op rate; the s_sleep kind
gives the board's power with every wave resident and no VALU issued.
    python tools/r4/valu_energy.py [--seconds 3] > out.json"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seconds", type=float, default=3.0)
ap.add_argument("--iters", type=int, default=4096)
ap.add_argument("--kinds", default="")
args = ap.parse_args()

lib = ctypes.CDLL(os.path.join(HERE, "libvalu_energy.so"))
lib.ve_name.restype = ctypes.c_char_p
lib.ve_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                          ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda", 0)
props = torch.cuda.get_device_properties(dev)
try:
    bdf = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}"
except AttributeError:
    bdf = ""
reader = bench.power_reader(bdf, 0)
blocks = props.multi_processor_count * 8          # 8 waves per SIMD
out_buf = torch.empty(blocks * 256, dtype=torch.int32, device=dev)
stamps = torch.zeros(blocks * 4, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
sync = torch.cuda.synchronize
kinds = [int(k) for k in args.kinds.split(",")] if args.kinds else list(range(lib.ve_kinds()))
res = {"blocks": blocks, "threads": 256, "iters": args.iters, "device": props.name, "kinds": {}}
for k in kinds:
    name = lib.ve_name(k).decode()
    step = lambda: lib.ve_launch(k, out_buf.data_ptr(), stamps.data_ptr(), blocks, args.iters, s)  # noqa: E731
    bench.settle(step, 300, sync)
    t0 = time.perf_counter()
    nl = 0
    while time.perf_counter() - t0 < 0.5:
        for _ in range(8):
            step()
        sync()
        nl += 8
    dt = (time.perf_counter() - t0) / nl
    pw = bench.power_probe(step, sync, args.seconds, reader)
    st = stamps.view(blocks, 4).cpu().numpy().astype(float)
    clk = statistics.median(((st[:, 2] - st[:, 0]) / (st[:, 3] - st[:, 1]) * 100.0).tolist())
    ops = blocks * 256 * args.iters * lib.ve_ops_per_iter(k)
    row = {"ms_per_launch": dt * 1e3, "in_kernel_clock_mhz": clk}
    if ops:
        row["t_lane_ops_per_s"] = ops / dt / 1e12
        row["cycles_per_wave_instr_per_simd"] = (dt * clk * 1e6) / (ops / 64 / (blocks * 4 // 8))
    if pw:
        row["power"] = pw
        w = pw.get("socket_power_w_median")
        if w and ops:
            row["pj_per_lane_op"] = w / (ops / dt) * 1e12
    res["kinds"][name] = row
    print(f"{name:36s} {dt*1e3:8.3f} ms  clk {clk:7.1f} MHz  "
          f"{row.get('t_lane_ops_per_s', 0):7.2f} T/s  "
          f"{(pw or {}).get('socket_power_w_median', 0):7.1f} W  {row.get('pj_per_lane_op', 0):6.2f} pJ",
          file=sys.stderr, flush=True)
base = res["kinds"].get("s_sleep (no VALU)", {}).get("power", {}).get("socket_power_w_median")
if base:
    for name, row in res["kinds"].items():
        w = row.get("power", {}).get("socket_power_w_median")
        if w and row.get("t_lane_ops_per_s"):
            row["pj_per_lane_op_above_sleep"] = (w - base) / (row["t_lane_ops_per_s"] * 1e12) * 1e12
print(json.dumps(res, indent=1))
