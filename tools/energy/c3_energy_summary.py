"""C3 energy budget (verdict r4 item 3): does static power x time + memory energy + the kernel
listing priced at measured per-instruction energies add up to the bench line's board energy per
product?  Inputs are one GPU session's files (round 5: tools/r5/gpu_r5b.sh, archived, tools/archive/MANIFEST.md) plus the C3 kernel's listing
(hipcc -S of csrc/kernels.hip, the library's code object):
    python tools/energy/c3_energy_summary.py gpurun_out/r5b build/kernels.s profiles/r5/c3_energy_budget.json
Every energy is 'above sleep': board power minus the power with every wave resident and sleeping,
per unit of work; the sleeping board (clock tree, leakage, fabric and HBM standby at that clock)
is charged as static power over the product's time.  The per-instruction energies come from
microbenchmarks running near 2.4 GHz; the product kernel runs at ~1.9 GHz under the 1,400 W cap
(lower voltage), so the listing's VALU energy is an upper bound at its clock; the report also
gives the compute-only ablation's energy (same instructions, no HBM traffic) as a cross-check."""
import collections
import json
import os
import re
import statistics
import sys

src, listing, dst = sys.argv[1], sys.argv[2], sys.argv[3]
KERNEL = "_ZN6nttmul6k_rowsINS_9Arith32P3EjjLi12ELi0ELb0E"
BATCH, N = 65536, 4096


def mix(path):
    s = open(path).read()
    m = re.search(r"^(%s\S*):" % re.escape(KERNEL), s, re.M)
    body = s[m.end():s.index(".Lfunc_end", m.end())]
    c = collections.Counter()
    for line in body.split("\n"):
        t = line.strip()
        if t and not t.startswith((".", ";")) and not t.endswith(":"):
            c[t.split()[0]] += 1
    return m.group(1), c


def classify(op):
    if op.startswith("v_mad_u64_u32") or op.startswith("v_mad_i64_i32"):
        return "v_mad_u64_u32"
    if op.startswith("v_mul_hi"):
        return "v_mul_hi_u32"
    if op.startswith("v_mul_lo"):
        return "v_mul_lo_u32"
    if op.startswith(("v_cndmask", "v_sub_co", "v_subrev_co", "v_add_co", "v_addc", "v_subb")):
        return "v_sub_co+v_cndmask (per instruction)"
    if op.startswith("v_"):
        return "simple"
    if op.startswith("ds_"):
        return "ds"
    return None


DS_DWORDS = {"ds_read2_b32": 2, "ds_write2_b32": 2, "ds_read_b32": 1, "ds_write_b32": 1,
             "ds_read_b64": 2, "ds_write_b64": 2, "ds_read2_b64": 4, "ds_write2_b64": 4}

name, c = mix(listing)
energy = json.load(open(os.path.join(src, "energy.json")))
d = energy["derived_above_sleep"]
pj = dict(d["pj_per_lane_op"])
pj["simple"] = statistics.mean(v for k, v in pj.items() if k in ("v_xor_b32", "v_add_u32"))
pj_ds = pj.get("ds_write_b32/ds_read_b32")
per_wave = collections.Counter()
for op, k in c.items():
    cl = classify(op)
    if cl == "ds":
        per_wave["ds dword-ops"] += k * DS_DWORDS.get(op, 1)
    elif cl:
        per_wave[cl] += k
waves = 4  # 256 threads per n = 4096 product
lanes = waves * 64
valu_uj = {cl: per_wave[cl] * lanes * pj[cl] * 1e-6 for cl in per_wave if cl != "ds dword-ops"}
lds_uj = per_wave["ds dword-ops"] * lanes * pj_ds * 1e-6 if pj_ds else None

line = json.loads(open(os.path.join(src, "c3_bench.json")).read().strip().splitlines()[-1])
pw = line["power"]
t_ns = line["roofline"]["kernel_ms"] * 1e6 / BATCH          # kernel time per product
board_uj = pw["board_uj_per_unit"]
sleep_w = d["sleep_w"]
static_uj = sleep_w * t_ns * 1e-3
rd, wr = d["pj_per_byte"]["hbm_read_16B_nt"], d["pj_per_byte"]["hbm_write_16B_nt"]
mem_uj = (2 * N * 4 * rd + N * 4 * wr) * 1e-6
l2_lane_bytes = (c.get("global_load_dwordx4", 0) * 16 + c.get("global_load_dwordx2", 0) * 8) * lanes
l2_uj = l2_lane_bytes * d["pj_per_byte"]["l2_read_16B"] * 1e-6
total = static_uj + mem_uj + sum(valu_uj.values()) + (lds_uj or 0) + l2_uj

# cross-check: kbench pricing variants of the same kernel, board energy per product
abl = {}
for v in ("base", "noload", "nostore", "noxchg", "compute"):
    f = os.path.join(src, "c3abl", v + ".smi.jsonl")
    out = os.path.join(src, "c3abl", v + ".out")
    if not os.path.exists(f):
        continue
    rows = []
    for ln in open(f):
        try:
            g = json.loads(ln)["gpu_data"][0]
        except (ValueError, KeyError, IndexError, TypeError):
            continue
        if (g["usage"]["gfx_activity"].get("value") or 0) >= 90:
            clk = [x["clk"]["value"] for k, x in g["clock"].items()
                   if k.startswith("gfx_") and isinstance(x.get("clk", {}).get("value"), (int, float))]
            rows.append((g["power"]["socket_power"]["value"], statistics.mean(clk) if clk else None))
    ms = float(open(out).read().split("ms")[0].split(":")[-1])
    if rows:
        w = statistics.median(r[0] for r in rows)
        abl[v] = {"ms": ms, "power_w": w, "clock_mhz": statistics.median(r[1] for r in rows if r[1]),
                  "uj_per_product": w * ms * 1e-3 / BATCH * 1e6, "samples": len(rows)}

# Closing the budget across operating points.  The per-instruction energies above come from
# microbenchmarks at ~2.3 GHz; the product kernel holds ~1.87 GHz under the 1,400 W cap, where the
# voltage (and so the dynamic energy per instruction) is lower.  One scale s(f) = 1 - k (F0 - f)
# for the compute side is fitted over the kbench variants of the same kernel, each at its own
# clock: E_v = sleep W x t_v + HBM(v) + s(f_v) x (D + LDS if it exchanges), with D = the
# compute-only variant's board energy above sleep at F0 (same instructions, twiddle loads kept,
# no a / b / c traffic, no exchanges) and HBM(v) = the variant's bytes at the stream energies.
F0 = abl["compute"]["clock_mhz"] / 1e3 if "compute" in abl else 2.38
D = (abl["compute"]["uj_per_product"] - sleep_w * abl["compute"]["ms"] * 1e-3 / BATCH * 1e6
     if "compute" in abl else None)
HBM = {"base": mem_uj, "noxchg": mem_uj, "noload": N * 4 * wr * 1e-6, "nostore": 2 * N * 4 * rd * 1e-6}
fit = None
if D:
    pts = []
    for v, h in HBM.items():
        if v not in abl:
            continue
        r = abl[v]
        dyn = D + (lds_uj if v != "noxchg" else 0)
        s_v = (r["uj_per_product"] - sleep_w * r["ms"] * 1e-3 / BATCH * 1e6 - h) / dyn
        pts.append((v, r["clock_mhz"] / 1e3, s_v, dyn, h, r))
    # least squares for k in 1 - s = k (F0 - f)
    num = sum((F0 - f) * (1 - sv) for _, f, sv, _, _, _ in pts)
    den = sum((F0 - f) ** 2 for _, f, sv, _, _, _ in pts)
    k = num / den
    sfun = lambda f: 1 - k * (F0 - f)  # noqa: E731
    fit = {"k_per_ghz": k, "F0_ghz": F0, "D_compute_uj_at_F0": D, "lds_uj_at_F0": lds_uj,
           "points": {v: {"clock_ghz": f, "s_needed": sv, "s_fit": sfun(f),
                          "measured_uj": r["uj_per_product"],
                          "model_uj": sleep_w * r["ms"] * 1e-3 / BATCH * 1e6 + h + sfun(f) * dyn,
                          } for v, f, sv, dyn, h, r in pts}}
    for p_ in fit["points"].values():
        p_["model_over_measured"] = p_["model_uj"] / p_["measured_uj"]
    # the C3 bench kernel at its held clock, broken down
    f_b = abl["base"]["clock_mhz"] / 1e3
    sb = sfun(f_b)
    listing = sum(valu_uj.values()) + l2_uj
    fit["base_breakdown_uj"] = {
        "static": sleep_w * abl["base"]["ms"] * 1e-3 / BATCH * 1e6,
        "hbm reads (32 KiB)": 2 * N * 4 * rd * 1e-6, "hbm writes (16 KiB)": N * 4 * wr * 1e-6,
        **{f"{k_} (share of D x s)": v * D / listing * sb for k_, v in valu_uj.items()},
        "l2 twiddle loads (share of D x s)": l2_uj * D / listing * sb,
        "lds exchanges (x s)": lds_uj * sb}
    fit["base_breakdown_uj"]["sum"] = sum(fit["base_breakdown_uj"].values())
    fit["base_breakdown_uj"]["measured"] = abl["base"]["uj_per_product"]
    # What 81.4 M/s at 1,400 W needs.  The compute side is issue-bound at its clock: time per
    # product = C (1 - x) / f for a cut x of the listing (count and energy alike); at the cap
    # 1400 = sleep + rate (HBM + s(f) (1 - x) Dtot).  Solve for the x at which the rate reaches
    # the target, and the HBM-byte cut y that would do it alone.
    Dtot = D + lds_uj
    C = abl["base"]["ms"] * 1e-3 / BATCH * f_b * 1e9           # cycles per product (chip-wide)
    target_rate = 81.4e6

    def power(x, y=0.0):
        f = target_rate * C * (1 - x) / 1e9                     # GHz the target rate needs
        return sleep_w + target_rate * 1e-6 * (mem_uj * (1 - y) + sfun(min(f, F0)) * (1 - x) * Dtot), f
    lo, hi = 0.0, 0.9
    for _ in range(60):
        mid = (lo + hi) / 2
        lo, hi = (mid, hi) if power(mid)[0] > 1400 else (lo, mid)
    fit["target"] = {"rate": target_rate, "uj_per_product_at_1400_w": 1400 / target_rate * 1e6,
                     "cycles_per_product_now": C, "valu_cut_needed_pct": hi * 100,
                     "clock_then_ghz": power(hi)[1],
                     "note": "the listing cut (instructions and their energy alike) at which 81.4 M "
                             "polymults/s fits in 1,400 W on the fitted s(f); HBM bytes are "
                             "algorithmic (48 KiB per product) and cannot be cut"}
out = {
    "kernel": name, "code_object": line["build"]["code_object"],
    "bench": {"value": line["value"], "kernel_ms": line["roofline"]["kernel_ms"],
              "board_uj_per_unit": board_uj, "socket_power_w": pw.get("socket_power_w_median"),
              "gfx_clock_mhz": pw.get("gfx_clock_mhz_median"),
              "in_kernel_clock_ghz": (line.get("in_kernel_clock") or {}).get("clock_ghz_median")},
    "per_wave_instructions": dict(per_wave),
    "pj_per_lane_op_above_sleep": pj, "pj_per_byte_above_sleep": d["pj_per_byte"],
    "sleep_w": sleep_w,
    "budget_uj_per_product": {
        "static (sleep power x kernel time per product)": static_uj,
        "hbm (32 KiB read + 16 KiB written, stream energies)": mem_uj,
        **{f"valu {k}": v for k, v in valu_uj.items()},
        "lds": lds_uj,
        "l2 twiddle loads (lane bytes, upper bound)": l2_uj,
        "sum": total,
        "measured (bench board_uj_per_unit)": board_uj,
        "sum / measured": total / board_uj},
    "ablations_kbench": abl,
    "operating_point_fit": fit,
    "source": f"{src}: energy.json (tools/energy/energy_microbench.py), c3_bench.json (bench.py), "
              "c3abl/ (kbench + amd-smi); listing: hipcc -S of csrc/kernels.hip",
}
os.makedirs(os.path.dirname(dst), exist_ok=True)
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out["budget_uj_per_product"], indent=1))
print(json.dumps(fit, indent=1))
