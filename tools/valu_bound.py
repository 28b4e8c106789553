"""VALU-issue bound of one kernel from its gfx950 ISA listing (the roofline that actually binds the
product kernel).

    python tools/valu_bound.py <kernels.s> <symbol-substring> <waves-per-launch> <clock-GHz> [kernel-ms]
        [--record N Q BATCH]

--record adds the result to profiles/valu_bound.json keyed by (N, Q) and the code object id of the
current lib/libnttmul.so (nttmul.code_object_id; build the listing from the same tree with
`make asm`), which bench.py looks up for its valu_roofline field.

cycles/wave = sum over the kernel's VALU instructions of the per-opcode SIMD issue cost measured
by tools/microbench/valu_issue.hip (cycles per wave64 instruction per SIMD, 8 waves/SIMD).
Instructions that write a carry or read a lane mask (v_*_co_*, v_addc/subb, v_cndmask, v_cmp) are
priced at CARRY_COST = 3.9 in either encoding (isolated VOP3 forms measure 4.1-4.4; the VCC e32
pair 2.4 only back to back without the 2-wait-state SGPR hazard), fitted on the compute-only
ablation (no loads, exchanges or stores; profiles/r1_ablation_clock.txt): 9,680 cycles per wave
measured, 9,709 predicted; the VCC-forced variant (cvcc) costs the same.  The bound is straight-line: every VALU
instruction of the listing runs once per wave (k_rows has no loops).
bound_ms = cycles/wave x waves per SIMD / clock.
"""
import collections
import json
import re
import sys

SIMDS = 1024  # 256 CUs x 4 SIMDs

# cycles per wave64 instruction per SIMD (tools/microbench/valu_issue.hip on MI355X)
COST = {
    "v_mad_u64_u32": 4.2, "v_mad_i64_i32": 4.2, "v_mul_lo_u32": 4.2, "v_mul_hi_u32": 4.2,
    "v_mul_u32_u24": 4.2, "v_mul_hi_u32_u24": 4.2, "v_min_u32": 4.2, "v_max_u32": 4.2,
    "v_med3_u32": 4.2, "v_lshlrev_b32": 4.2, "v_add3_u32": 4.2, "v_lshl_add_u32": 4.2,
    "v_lshl_add_u64": 4.2, "v_cmp_ge_u64": 4.2, "v_cmp_gt_u64": 4.2, "v_cmp_lt_u64": 4.2,
    "v_cmp_eq_u64": 4.2, "v_cmp_ne_u64": 4.2, "v_lshlrev_b64": 4.2, "v_lshrrev_b64": 4.2,
    "v_fma_f32": 3.8,
}
CHEAP = 2.3  # v_add/sub, logic, shifts right, moves
# carry-writing / mask-reading instructions: fitted so the compute-only ablation's listing
# predicts its measured 9,680 cycles per wave (9,709 at 3.9)
CARRY_COST = 3.9


CARRY = re.compile(r"^v_(add|sub|subrev)_co_|^v_(addc|subb|subbrev)_co_|^v_cndmask_|^v_cmp")


def cost(op: str) -> float:
    base = re.sub(r"_e(32|64)$", "", op)
    if CARRY.match(base):
        return CARRY_COST
    return COST.get(base, CHEAP)


def main():
    argv = sys.argv[1:]
    record = None
    if "--record" in argv:
        i = argv.index("--record")
        record = [int(x) for x in argv[i + 1:i + 4]]
        argv = argv[:i] + argv[i + 4:]
    path, key, waves, ghz = argv[0], argv[1], int(argv[2]), float(argv[3])
    kms = float(argv[4]) if len(argv) > 4 else None
    s = open(path).read()
    m = re.search(r"^(\S*%s\S*):\s*;" % re.escape(key), s, re.M)
    body = s[m.end():s.index(".Lfunc_end", m.end())]
    ops = [ln.strip().split()[0] for ln in body.split("\n")
           if ln.strip().startswith("v_")]
    hist = collections.Counter(ops)
    cyc = sum(cost(o) * c for o, c in hist.items())
    per_simd = waves / SIMDS
    bound_ms = cyc * per_simd / (ghz * 1e9) * 1e3
    out = {"kernel": m.group(1), "valu_per_wave": len(ops), "cycles_per_wave": round(cyc, 1),
           "waves_per_simd": per_simd, "clock_ghz": ghz, "valu_bound_ms": round(bound_ms, 4)}
    if kms:
        out["kernel_ms"] = kms
        out["frac_of_valu_bound"] = round(bound_ms / kms, 4)
    out["top"] = {o: c for o, c in hist.most_common(12)}
    if record:
        import os
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, os.path.join(root, "ntt-based-polynomial-multiplier-fpga_amd"))
        import nttmul
        out.update(n=record[0], q=record[1], batch=record[2],
                   code_object=nttmul.code_object_id(),
                   source="tools/valu_bound.py on `make asm` (build/kernels.s) of this tree")
        tpath = os.path.join(root, "profiles", "valu_bound.json")
        table = json.load(open(tpath)) if os.path.exists(tpath) else {"entries": []}
        table["entries"] = [e for e in table["entries"]
                            if not (e["n"] == out["n"] and e["q"] == out["q"]
                                    and e.get("code_object") == out["code_object"])]
        table["entries"].append(out)
        json.dump(table, open(tpath, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
