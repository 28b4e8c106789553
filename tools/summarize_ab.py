"""Summarise a tools/kbench/ab_power.sh directory: per variant and round, the kbench timing line
(time per launch, output checksum) and the medians of the amd-smi samples taken while it ran
(gfx-busy samples: socket power, shader clock, UMC activity, PPT violation count).

    python tools/summarize_ab.py <ab dir> [out.json]
"""
import glob
import json
import os
import re
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_power import sample  # noqa: E402


def main():
    src = sys.argv[1]
    out = {}
    for f in sorted(glob.glob(os.path.join(src, "r*", "*.out"))):
        rnd = os.path.basename(os.path.dirname(f))
        v = os.path.basename(f)[:-4]
        line = open(f).read().strip()
        m = re.search(r":\s*([\d.]+) ms.*chk=(\w+)", line)
        rows = []
        for ln in open(f[:-4] + ".smi.jsonl"):
            try:
                rows.append(sample(json.loads(ln)))
            except (ValueError, KeyError, IndexError, TypeError):
                continue
        busy = [r for r in rows if (r["gfx_activity_pct"] or 0) >= 90 and r["socket_power_w"]]

        def med(k):
            xs = [r[k] for r in busy if isinstance(r.get(k), (int, float))]
            return statistics.median(xs) if xs else None
        out.setdefault(v, []).append({
            "round": rnd, "ms": float(m.group(1)) if m else None, "checksum": m.group(2) if m else None,
            "busy_samples": len(busy), "socket_power_w": med("socket_power_w"),
            "gfx_clock_mhz": med("gfx_clk_mhz"), "umc_activity_pct": med("umc_activity_pct"),
            "ppt_violation_samples": sum(1 for r in busy if r.get("ppt_violation") in (True, 1, "ACTIVE")),
            "line": line})
    summary = {v: {"ms": [r["ms"] for r in rs], "mean_ms": statistics.mean(r["ms"] for r in rs),
                   "checksums": sorted({r["checksum"] for r in rs}),
                   "power_w": [r["socket_power_w"] for r in rs],
                   "gfx_clock_mhz": [r["gfx_clock_mhz"] for r in rs]} for v, rs in out.items()}
    res = {"source": src, "summary": summary, "runs": out}
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
