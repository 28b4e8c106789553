"""VALU-issue bound of a product step's kernels from their gfx950 ISA listings (the roofline that
actually binds the product kernels).

    python tools/valu_bound.py <kernels.s> N Q BATCH "<dispatch names>" [--kernel-ms MS] [--record]

<dispatch names> is the step's nttmul_kernel_name string, e.g. "k_rows<Arith32P3,u32,u32,12,0>"
(C3) or "k_cols8<Arith64,u64,fwd> + k_rows<Arith64,u64,u64,8,8> + k_cols8<Arith64,u64,inv>" (C5);
build the listing from the same tree with `make -C ntt-based-polynomial-multiplier-fpga_amd asm`.
--record adds the result to profiles/valu_bound.json keyed by (N, Q) and the per-kernel hashes of
the current lib/libnttmul.so (nttmul.kernel_hashes), which bench.py looks up for its
valu_roofline field: an entry stays valid while those kernels' machine code does.

cycles/wave = sum over the kernel's VALU instructions of the per-opcode SIMD issue cost measured
by tools/microbench/valu_issue.hip (cycles per wave64 instruction per SIMD, 8 waves/SIMD).
Instructions that write a carry or read a lane mask (v_*_co_*, v_addc/subb, v_cndmask, v_cmp) are
priced at CARRY_COST = 3.9 in either encoding (isolated VOP3 forms measure 4.1-4.4; the VCC e32
pair 2.4 only back to back without the 2-wait-state SGPR hazard), fitted on the compute-only
ablation (no loads, exchanges or stores; profiles/r1_ablation_clock.txt): 9,680 cycles per wave
measured, 9,709 predicted.  The bound is straight-line: every VALU instruction of the listing runs
once per wave; the tool refuses a kernel whose listing has a backward branch (a loop).
waves per polynomial: every product kernel gives a thread 16 coefficients (k_rows, k_cols8) or
one column of 2^L1 (k_cols_fwd / k_cols_inv), so n / 1024 or n / 2^L1 / 64 waves.
bound_ms = sum over kernels of cycles/wave x waves per SIMD / clock.
"""
import collections
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd"))
import nttmul  # noqa: E402

SIMDS = 1024  # 256 CUs x 4 SIMDs
MAX_CLOCK_GHZ = 2.4

# cycles per wave64 instruction per SIMD (tools/microbench/valu_issue.hip on MI355X)
COST = {
    "v_mad_u64_u32": 4.2, "v_mad_i64_i32": 4.2, "v_mul_lo_u32": 4.2, "v_mul_hi_u32": 4.2,
    "v_mul_hi_i32": 4.2, "v_mul_u32_u24": 4.2, "v_mul_hi_u32_u24": 4.2, "v_min_u32": 4.2,
    "v_max_u32": 4.2, "v_med3_u32": 4.2, "v_lshlrev_b32": 4.2, "v_add3_u32": 4.2,
    "v_lshl_add_u32": 4.2, "v_lshl_add_u64": 4.2, "v_cmp_ge_u64": 4.2, "v_cmp_gt_u64": 4.2,
    "v_cmp_lt_u64": 4.2, "v_cmp_eq_u64": 4.2, "v_cmp_ne_u64": 4.2, "v_lshlrev_b64": 4.2,
    "v_lshrrev_b64": 4.2, "v_fma_f32": 3.8,
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


def waves_per_unit(key: str, n: int) -> float:
    """Waves one polynomial product takes in this kernel (see the module docstring)."""
    kern, args = key.split("<", 1)
    args = args.rstrip(">").split(",")
    if kern in ("k_rows", "k_cols8"):
        return n / 16 / 64
    if kern in ("k_cols_fwd", "k_cols_inv"):
        return n / (1 << int(args[2])) / 64
    raise ValueError(f"no wave count rule for {key}")


def listing_body(s: str, key: str):
    """(symbol, body text) of the kernel whose kernel_key is `key` in a `make asm` listing."""
    for m in re.finditer(r"^(_ZN6nttmul\S*):\s*;", s, re.M):
        if nttmul.kernel_key(m.group(1)) == key:
            return m.group(1), s[m.end():s.index(".Lfunc_end", m.end())]
    raise KeyError(f"{key} not in the listing")


def kernel_bound(s: str, key: str, n: int) -> dict:
    sym, body = listing_body(s, key)
    lines = [ln.strip() for ln in body.split("\n")]
    labels = {ln[:-1] for ln in lines if re.match(r"^\.LBB\S+:$", ln)}
    seen, back = set(), []
    for ln in lines:
        if ln[:-1] in labels:
            seen.add(ln[:-1])
        elif ln.startswith(("s_branch", "s_cbranch")) and ln.split()[-1] in seen:
            back.append(ln)
    if back:
        raise ValueError(f"{key}: loop in the listing ({back[0]}): the straight-line bound does not apply")
    ops = [ln.split()[0] for ln in lines if ln.startswith("v_")]
    hist = collections.Counter(ops)
    return {"kernel": key, "symbol": sym, "valu_per_wave": len(ops),
            "cycles_per_wave": round(sum(cost(o) * c for o, c in hist.items()), 1),
            "waves_per_unit": waves_per_unit(key, n),
            "top": dict(hist.most_common(12))}


def main():
    argv = sys.argv[1:]
    record = "--record" in argv
    argv = [a for a in argv if a != "--record"]
    kms = None
    if "--kernel-ms" in argv:
        i = argv.index("--kernel-ms")
        kms = float(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    path, n, q, batch, names = argv[0], int(argv[1]), int(argv[2]), int(argv[3]), argv[4]
    s = open(path).read()
    keys = [nttmul.dispatch_key(x) for x in names.split("+")]
    per = [kernel_bound(s, k, n) for k in keys]
    cycles_per_unit = sum(p["cycles_per_wave"] * p["waves_per_unit"] for p in per)
    bound_ms = cycles_per_unit * batch / SIMDS / (MAX_CLOCK_GHZ * 1e9) * 1e3
    out = {"n": n, "q": q, "batch": batch, "dispatch": names.strip(),
           "kernels": nttmul.dispatched_kernel_hashes(names),
           "per_kernel": per, "cycles_per_unit": round(cycles_per_unit, 1),
           "clock_ghz": MAX_CLOCK_GHZ, "valu_bound_ms": round(bound_ms, 4),
           "code_object": nttmul.code_object_id(),
           "source": "tools/valu_bound.py on `make asm` (build/kernels.s) of this tree"}
    if kms:
        out["kernel_ms"] = kms
        out["frac_of_valu_bound"] = round(bound_ms / kms, 4)
    if record:
        tpath = os.path.join(ROOT, "profiles", "valu_bound.json")
        table = json.load(open(tpath)) if os.path.exists(tpath) else {"entries": []}
        table["entries"] = [e for e in table["entries"]
                            if not (e["n"] == n and e["q"] == q and e.get("kernels") == out["kernels"])]
        table["entries"].append(out)
        json.dump(table, open(tpath, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
