"""Board energy of each work class in the C3 product kernel (verdict r4 item 3), measured on the
GPU box: every kind of tools/energy/energy.hip runs back to back for --seconds while bench.power_probe
samples socket power in process (amdsmi), the rate comes from wall time over the same launches
and the clock from the kernel's own s_memtime / s_memrealtime stamps.  Reports per kind the board
power, the clock, and energies above the all-waves-sleeping board power:
  VALU: pJ per lane-op of the instruction itself (the pair kinds minus their xor refresh),
  LDS:  pJ per lane-op of ds_write_b32 / ds_read_b32 (their xor removed),
  memory: pJ per byte read / written / copied from HBM, per byte read from L2.
    python tools/energy/energy_microbench.py [--seconds 3] > energy.json   (build libenergy.so first:
    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/energy/energy.hip -o tools/energy/libenergy.so)"""
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
ap.add_argument("--kinds", default="")
args = ap.parse_args()

lib = ctypes.CDLL(os.path.join(HERE, "libenergy.so"))
lib.en_name.restype = ctypes.c_char_p
lib.en_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                          ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                          ctypes.c_void_p]
dev = torch.device("cuda", 0)
props = torch.cuda.get_device_properties(dev)
try:
    bdf = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}"
except AttributeError:
    bdf = ""
reader = bench.power_reader(bdf, 0)
blocks = props.multi_processor_count * 8          # 8 waves per SIMD (2048 on MI355X: 2^19 lanes)
n16 = 1 << 27                                     # 2 GiB of 16-byte words per buffer
out_buf = torch.empty(blocks * 256, dtype=torch.int32, device=dev)
stamps = torch.zeros(blocks * 4, dtype=torch.int64, device=dev)
src = torch.randint(0, 1 << 30, (n16 * 4,), dtype=torch.int32, device=dev)
dst = torch.empty_like(src)
s = torch.cuda.current_stream(dev).cuda_stream
sync = torch.cuda.synchronize
names = [lib.en_name(k).decode() for k in range(lib.en_kinds())]
kinds = [int(k) for k in args.kinds.split(",")] if args.kinds else list(range(lib.en_kinds()))
ITERS = {"sleep": 4096, "hbm_read_16B_nt": 128, "hbm_write_16B_nt": 128, "hbm_copy_16B_nt": 64,
         "l2_read_16B": 4096, "ds_write_b32+ds_read_b32+xor": 2048}
res = {"blocks": blocks, "threads": 256, "device": props.name,
       "source": "tools/energy/energy.hip kinds, board power by amdsmi in process (bench.power_probe)",
       "kinds": {}}
for k in kinds:
    name = names[k]
    iters = ITERS.get(name, 4096)
    step = lambda: lib.en_launch(k, out_buf.data_ptr(), stamps.data_ptr(), src.data_ptr(),  # noqa: E731
                                 dst.data_ptr(), n16, blocks, iters, s)
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
    lanes = blocks * 256 * iters
    row = {"iters": iters, "ms_per_launch": dt * 1e3, "in_kernel_clock_mhz": clk,
           "valu_lane_ops_per_s": lanes * lib.en_valu_per_iter(k) / dt,
           "lds_lane_ops_per_s": lanes * lib.en_lds_per_iter(k) / dt,
           "bytes_per_s": lanes * lib.en_bytes_per_iter(k) / dt}
    if pw:
        row["power"] = pw
    res["kinds"][name] = row
    print(f"{name:34s} {dt * 1e3:8.3f} ms  clk {clk:7.1f} MHz  "
          f"{(pw or {}).get('socket_power_w_median', 0):7.1f} W  "
          f"{row['bytes_per_s'] / 1e12:6.2f} TB/s", file=sys.stderr, flush=True)


def watts(name):
    return res["kinds"].get(name, {}).get("power", {}).get("socket_power_w_median")


base = watts("sleep")
derived = {"sleep_w": base}
if base:
    def above(name, rate_key):
        w, r = watts(name), res["kinds"].get(name, {}).get(rate_key)
        return (w - base) / r * 1e12 if w and r else None
    xor = above("v_xor_b32", "valu_lane_ops_per_s")        # pJ per xor lane-op
    derived["pj_per_lane_op"] = {"v_xor_b32": xor, "v_add_u32": above("v_add_u32", "valu_lane_ops_per_s")}
    for name, key, per in (("v_mul_hi_u32+xor", "v_mul_hi_u32", 2), ("v_mul_lo_u32+xor", "v_mul_lo_u32", 2),
                           ("v_mad_u64_u32+xor", "v_mad_u64_u32", 2),
                           ("v_sub_co+v_cndmask+xor", "v_sub_co+v_cndmask (per instruction)", 3)):
        e = above(name, "valu_lane_ops_per_s")
        if e is not None and xor is not None:  # (per ops x average - one xor) / the others' count
            derived["pj_per_lane_op"][key] = (per * e - xor) / (per - 1)
    e = above("ds_write_b32+ds_read_b32+xor", "lds_lane_ops_per_s")
    w = watts("ds_write_b32+ds_read_b32+xor")
    kk = res["kinds"].get("ds_write_b32+ds_read_b32+xor", {})
    if w and xor is not None and kk.get("lds_lane_ops_per_s"):
        # power above sleep minus the xors' share, per LDS lane-op
        derived["pj_per_lane_op"]["ds_write_b32/ds_read_b32"] = (
            (w - base) - xor * 1e-12 * kk["valu_lane_ops_per_s"]) / kk["lds_lane_ops_per_s"] * 1e12
    derived["pj_per_byte"] = {k: above(k, "bytes_per_s") for k in
                              ("hbm_read_16B_nt", "hbm_write_16B_nt", "hbm_copy_16B_nt", "l2_read_16B")}
res["derived_above_sleep"] = derived
print(json.dumps(res, indent=1))
