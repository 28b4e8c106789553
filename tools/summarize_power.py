"""Summarise a tools/gpu_power.sh session (amd-smi samples taken while each workload ran).

    python tools/summarize_power.py gpurun_out/power profiles/r2/power

Writes <dst>/samples.json (per label: socket power, mean shader clock over the 8 XCDs, hotspot
temperature, gfx / UMC activity and the PPT (package power) violation flag of every sample) and
<dst>/summary.json (per label: medians over the busy samples, gfx activity >= 90 %, plus the
workload's own timing line).
"""
import glob
import json
import os
import statistics
import sys


def val(x):
    return x.get("value") if isinstance(x, dict) else None


def sample(doc):
    g = doc["gpu_data"][0] if isinstance(doc, dict) else doc[0]
    clk = [val(v.get("clk", {})) for k, v in g["clock"].items() if k.startswith("gfx_")]
    clk = [c for c in clk if isinstance(c, (int, float))]
    th = g.get("throttle", {})
    return {
        "socket_power_w": val(g["power"]["socket_power"]),
        "gfx_clk_mhz": round(sum(clk) / len(clk), 1) if clk else None,
        "hotspot_c": val(g["temperature"].get("hotspot", {})),
        "gfx_activity_pct": val(g["usage"]["gfx_activity"]),
        "umc_activity_pct": val(g["usage"]["umc_activity"]),
        "ppt_violation": th.get("ppt_violation_status"),
    }


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    samples, summary = {}, {}
    if os.path.exists(os.path.join(src, "static.json")):  # (tools/gpu_power.sh records it)
        static = json.load(open(os.path.join(src, "static.json")))
        lim = static["gpu_data"][0]["limit"]["ppt0"]["socket_power_limit"]
        summary["socket_power_limit_w"] = val(lim)
    for f in sorted(glob.glob(os.path.join(src, "*.smi.jsonl"))):
        label = os.path.basename(f)[: -len(".smi.jsonl")]
        rows = []
        for line in open(f):
            line = line.strip()
            if not line:
                continue
            try:
                rows.append(sample(json.loads(line)))
            except (ValueError, KeyError, IndexError, TypeError):
                continue
        samples[label] = rows
        busy = [r for r in rows if (r["gfx_activity_pct"] or 0) >= 90]
        out = open(os.path.join(src, label + ".out")).read().strip().splitlines()
        s = {"samples": len(rows), "busy_samples": len(busy), "timing": out[-1] if out else None}
        if busy:
            for k in ("socket_power_w", "gfx_clk_mhz", "hotspot_c", "umc_activity_pct"):
                s["median_" + k] = statistics.median(r[k] for r in busy)
            s["ppt_violation_active"] = sum(r["ppt_violation"] == "ACTIVE" for r in busy)
        summary[label] = s
    json.dump(samples, open(os.path.join(dst, "samples.json"), "w"), indent=1)
    json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
