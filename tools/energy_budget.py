"""C5 energy budget (verdict r5 item 2b): static power x time + HBM bytes at the measured per-byte
energies + the three kernels' listings at the measured per-instruction energies, with one
voltage scale s(f) for the compute side, fitted over the round-5 C5 pricing variants (the same
instruction streams with the intermediates' loads and / or stores redirected on chip, each at its
own clock and power) and checked against the bench line's board energy per product.

    python tools/energy_budget.py --listing-fit <r5 listing .s> --listing <listing .s> \\
        --bench <c5 bench.json> [--out profiles/r6/c5_energy_budget.json]

Inputs (all committed or rebuildable):
  profiles/r5/energy/energy.json            per-op energies above the sleeping board (357 W),
                                            HBM read / write and L2 stream energies per byte
  profiles/r5/c5_split/power_session_b_c5ab{1,2}.json   the t_* variants (square split, tiled
                                            intermediates = the library's C5): time, median
                                            socket power, gfx clock, UMC activity per run
  --listing-fit   `hipcc -S` of the round-5 kernels the variants ran (commit 97692dc)
  --listing       the listing of the kernels the bench line ran (`make asm` of this tree)
HBM bytes per product of a variant: the bytes it still sends to memory (base: the PMC-measured
4.72 MB, 2.5 MiB read and 2 MiB written); the redirected intermediates are charged at the L2
stream energy.  Energies are per product, in uJ."""
import argparse
import collections
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd"))
import nttmul  # noqa: E402

BATCH = 1024
N = 65536
KERNELS = ["k_cols8<Arith64,u64,u64,0,2>", "k_rows<Arith64,u64,u64,8,8,false>",
           "k_cols8<Arith64,u64,u64,1,1>"]
LANES = N // 16  # every C5 kernel gives a thread 16 coefficients: 4,096 lanes per product
READ_B, WRITE_B = 5 * N * 8, 4 * N * 8  # 2.5 MiB read (a, b, ta, tb, tc), 2 MiB written (ta, tb, tc, c)
LDS_DWORDS = {"ds_read2_b32": 2, "ds_write2_b32": 2, "ds_read_b32": 1, "ds_write_b32": 1,
              "ds_read_b64": 2, "ds_write_b64": 2, "ds_read2_b64": 4, "ds_write2_b64": 4,
              "ds_read2st64_b64": 4, "ds_write2st64_b64": 4}


def classify(op):
    if op.startswith(("v_mad_u64_u32", "v_mad_i64_i32")):
        return "v_mad_u64_u32"
    if op.startswith("v_mul_hi"):
        return "v_mul_hi_u32"
    if op.startswith("v_mul_lo"):
        return "v_mul_lo_u32"
    if op.startswith(("v_cndmask", "v_sub_co", "v_subrev_co", "v_add_co", "v_addc", "v_subb",
                      "v_cmp")):
        return "carry/select"
    if op.startswith("v_"):
        return "simple"
    if op.startswith("ds_"):
        return "lds"
    return None


def mixes(listing):
    """{kernel key: Counter of instruction classes (LDS as dword-ops)} for the C5 kernels."""
    s = open(listing).read()
    out = {}
    for m in re.finditer(r"^(_ZN6nttmul\S*):\s*;", s, re.M):
        key = nttmul.kernel_key(m.group(1))
        if key not in KERNELS:
            continue
        body = s[m.end():s.index(".Lfunc_end", m.end())]
        c = collections.Counter()
        for ln in body.split("\n"):
            t = ln.strip()
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            op = t.split()[0]
            cl = classify(op)
            if cl == "lds":
                c["lds dword-ops"] += LDS_DWORDS.get(op, 1)
            elif cl:
                c[cl] += 1
        out[key] = c
    missing = [k for k in KERNELS if k not in out]
    if missing:
        raise SystemExit(f"{listing}: no {missing}")
    return out


def compute_uj(mix, pj):
    """Listing energy per product at the microbenchmarks' clock (F0), above sleep."""
    per = {}
    for k, c in mix.items():
        e = sum(n * pj[cl] for cl, n in c.items())
        per[k] = e * LANES * 1e-6
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--listing-fit", required=True)
    ap.add_argument("--listing", required=True)
    ap.add_argument("--bench", required=True)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r6", "c5_energy_budget.json"))
    a = ap.parse_args()
    en = json.load(open(os.path.join(ROOT, "profiles", "r5", "energy", "energy.json")))
    d = en["derived_above_sleep"]
    sleep_w = d["sleep_w"]
    pj = {"v_mad_u64_u32": d["pj_per_lane_op"]["v_mad_u64_u32"],
          "v_mul_hi_u32": d["pj_per_lane_op"]["v_mul_hi_u32"],
          "v_mul_lo_u32": d["pj_per_lane_op"]["v_mul_lo_u32"],
          "carry/select": d["pj_per_lane_op"]["v_sub_co+v_cndmask (per instruction)"],
          "simple": statistics.mean([d["pj_per_lane_op"]["v_xor_b32"], d["pj_per_lane_op"]["v_add_u32"]]),
          "lds dword-ops": d["pj_per_lane_op"]["ds_write_b32/ds_read_b32"]}
    rd, wr = d["pj_per_byte"]["hbm_read_16B_nt"], d["pj_per_byte"]["hbm_write_16B_nt"]
    l2 = d["pj_per_byte"]["l2_read_16B"]
    hbm_base = (READ_B * rd + WRITE_B * wr) * 1e-6
    hbm_pj_per_b = (READ_B * rd + WRITE_B * wr) / (READ_B + WRITE_B)
    # F0: the clock the per-op microbenchmarks ran at (energy.json's VALU kinds, in-kernel)
    F0 = statistics.median(k["in_kernel_clock_mhz"] for n_, k in en["kinds"].items()
                           if n_.startswith("v_")) / 1e3

    mix_fit = mixes(a.listing_fit)
    comp_fit = compute_uj(mix_fit, pj)
    C_fit = sum(comp_fit.values())

    # the round-5 variants (two interleaved sessions).  HBM bytes per product: the nominal bytes
    # each variant still sends to memory (the redirected intermediates charged at the L2 stream
    # energy instead); the UMC-activity-scaled estimate is reported beside it
    nominal = {"t_base": (READ_B, WRITE_B), "t_st": (READ_B, N * 8),
               "t_ld": (2 * N * 8, WRITE_B), "t_ldst": (2 * N * 8, N * 8), "t_all": (0, N * 8)}
    pts = []
    for sess in (1, 2):
        data = json.load(open(os.path.join(ROOT, "profiles", "r5", "c5_split",
                                           f"power_session_b_c5ab{sess}.json")))
        base = data["t_base"]
        tb = float(base["timing"].split(":")[1].split("ms")[0])
        for v, (rb, wb) in nominal.items():
            r = data[v]
            t = float(r["timing"].split(":")[1].split("ms")[0])
            umc_bytes = (READ_B + WRITE_B) * (r["median_umc_activity_pct"] * t) / (
                base["median_umc_activity_pct"] * tb)
            e_meas = r["median_socket_power_w"] * t * 1e-3 / BATCH * 1e6
            static = sleep_w * t * 1e-3 / BATCH * 1e6
            e_hbm = (rb * rd + wb * wr) * 1e-6
            e_l2 = (READ_B + WRITE_B - rb - wb) * l2 * 1e-6
            pts.append({"variant": v, "session": sess, "ms": t, "power_w": r["median_socket_power_w"],
                        "gfx_clock_ghz": r["median_gfx_clk_mhz"] / 1e3,
                        "umc_pct": r["median_umc_activity_pct"], "hbm_bytes_nominal": rb + wb,
                        "hbm_bytes_umc_scaled": umc_bytes, "measured_uj": e_meas,
                        "static_uj": static, "hbm_uj": e_hbm, "onchip_uj": e_l2,
                        "compute_needed_uj": e_meas - static - e_hbm - e_l2})
    # Model A (used): compute = s x listing energy, one constant s for the mixed instruction
    # stream (the per-op energies come from single-instruction loops at F0), fitted as the mean
    # over the ten runs.  Model B (diagnostic): C3's linear voltage scale s(f) = 1 - k (F0 - f),
    # k fitted by least squares; the C5 variants do not follow it (their compute_needed is flat
    # over 1.95-2.37 GHz), see the residuals.
    s_const = statistics.mean(p["compute_needed_uj"] / C_fit for p in pts)
    xs = [(F0 - p["gfx_clock_ghz"]) for p in pts]
    ys = [1 - p["compute_needed_uj"] / C_fit for p in pts]
    k = sum(x * y for x, y in zip(xs, ys)) / sum(x * x for x in xs)
    for p in pts:
        p["s_needed"] = p["compute_needed_uj"] / C_fit
        p["model_uj"] = p["static_uj"] + p["hbm_uj"] + p["onchip_uj"] + s_const * C_fit
        p["model_over_measured"] = p["model_uj"] / p["measured_uj"]
        p["model_b_over_measured"] = (p["static_uj"] + p["hbm_uj"] + p["onchip_uj"] +
                                      (1 - k * (F0 - p["gfx_clock_ghz"])) * C_fit) / p["measured_uj"]

    def s(f):  # model A: no clock dependence
        return s_const
    # the bench line of this tree
    line = json.loads(open(a.bench).read().strip().splitlines()[-1])
    pw = line["power"]
    f_b = pw["gfx_clock_mhz_median"] / 1e3
    t_ns = line["roofline"]["kernel_ms"] * 1e6 / BATCH
    mix_b = mixes(a.listing)
    comp_b = compute_uj(mix_b, pj)
    sb = s(f_b)
    budget = {"static (357 W sleeping board x kernel time per product)": sleep_w * t_ns * 1e-3,
              "hbm reads (2.5 MiB: a, b and the three intermediates' reads)": READ_B * rd * 1e-6,
              "hbm writes (2 MiB: ta, tb, tc and c)": WRITE_B * wr * 1e-6}
    for kk, v in comp_b.items():
        budget[f"compute {kk} (listing x per-op energies x s(f))"] = v * sb
    budget["sum"] = sum(budget.values())
    budget["measured (bench board_uj_per_unit)"] = pw["board_uj_per_unit"]
    budget["sum / measured"] = budget["sum"] / pw["board_uj_per_unit"]
    # the largest compute terms, per product, priced at the bench clock
    terms = collections.Counter()
    for kk, c in mix_b.items():
        for cl, n in c.items():
            terms[f"{kk}: {cl}"] = n * pj[cl] * LANES * 1e-6 * sb
    # what the intermediates are worth in energy, and the floor with them on chip
    inter_b = (1.5 * 2 ** 20 * rd + 1.5 * 2 ** 20 * wr) * 1e-6
    # time per product at the cap: (HBM + compute) / (cap - sleep); static is paid per time
    cap = pw.get("socket_power_cap_w") or 1400.0
    comp_now = sum(comp_b.values()) * sb
    alg = (2 * N * 8 * rd + N * 8 * wr) * 1e-6
    floor = {}
    for name, hb, cp in (("this listing, every byte", hbm_base, comp_now),
                         ("this listing, intermediates free (algorithmic 1.5 MiB only)", alg, comp_now),
                         ("no HBM energy at all (compute only)", 0.0, comp_now)):
        us = (hb + cp) / (cap - sleep_w)
        floor[name] = {"us_per_product": us, "ms_per_batch": us * BATCH / 1e3,
                       "m_polymults_per_s": 1.0 / us, "hbm_roofline_frac": (3 * N * 8) / (us * 1e-6) / 8e12}
    us50 = 3 * N * 8 / 4e12 * 1e6
    floor["north-star 50 % needs"] = {
        "us_per_product": us50,
        "compute_uj_allowed_with_algorithmic_hbm": us50 * (cap - sleep_w) - alg,
        "compute_uj_now": comp_now,
        "note": "the compute energy per product that would fit 50 % of the HBM roofline at the cap "
                "with only the algorithmic 1.5 MiB moved"}
    out = {
        "config": "C5: n = 65536, q = 4611686018425815041, batch 1024 (square split, three launches)",
        "bench": {"value": line["value"], "kernel_ms": line["roofline"]["kernel_ms"],
                  "board_uj_per_unit": pw["board_uj_per_unit"], "socket_power_w": pw.get("socket_power_w_median"),
                  "gfx_clock_mhz": pw.get("gfx_clock_mhz_median"),
                  "in_kernel_clock_ghz": (line.get("in_kernel_clock") or {}).get("clock_ghz_median"),
                  "kernels": line.get("build", {}).get("kernels")},
        "per_op_pj_above_sleep": pj, "hbm_pj_per_byte": {"read": rd, "write": wr}, "l2_pj_per_byte": l2,
        "sleep_w": sleep_w, "F0_ghz": F0,
        "listing_bench": {k_: dict(v) for k_, v in mix_b.items()},
        "listing_fit_r5": {k_: dict(v) for k_, v in mix_fit.items()},
        "compute_at_F0_uj": {"fit listing (r5 kernels)": C_fit, "bench listing": sum(comp_b.values()),
                             **{f"bench {k_}": v for k_, v in comp_b.items()}},
        "mixed_stream_scale": {
            "s": s_const, "model_over_measured_range": [min(p["model_over_measured"] for p in pts),
                                                        max(p["model_over_measured"] for p in pts)],
            "linear_voltage_fit_k_per_ghz": k,
            "linear_fit_residual_range": [min(p["model_b_over_measured"] for p in pts),
                                          max(p["model_b_over_measured"] for p in pts)],
            "note": "model A (used): compute = s x listing at the per-op energies, s constant; "
                    "model B: s(f) = 1 - k (F0 - f) as in the C3 budget -- the C5 variants' compute "
                    "energy is flat over 1.95-2.37 GHz, so B misfits the on-chip variants"},
        "variants_r5": pts,
        "budget_uj_per_product": budget,
        "largest_compute_terms_uj": dict(terms.most_common(8)),
        "floor_at_the_cap": floor,
        "intermediates": {"hbm_uj_per_product": inter_b,
                          "share_of_measured": inter_b / pw["board_uj_per_unit"],
                          "note": "1.5 MiB written (ta, tb, tc) and read back per product"},
        "source": "tools/energy_budget.py: profiles/r5/energy/energy.json, "
                  "profiles/r5/c5_split/power_session_b_c5ab{1,2}.json, listings by hipcc -S",
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({"budget": budget, "s": s_const, "k": k, "F0": F0, "C_fit": C_fit,
                      "variants": [(p["variant"], p["session"], round(p["model_over_measured"], 3),
                                    round(p["model_b_over_measured"], 3)) for p in pts],
                      "terms": out["largest_compute_terms_uj"], "floor": floor}, indent=1))


if __name__ == "__main__":
    main()
