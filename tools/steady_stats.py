"""Per-kernel durations from a rocprofv3 kernel trace, split into the whole run and its last K
dispatches of each kernel (bench.py's timed steps come last: the settle and warm-up launches,
including the first ≈ 40 ms of the card's clock ramp, come before them).  rocprofv3's
--stats average covers every dispatch, ramp included; this gives the steady-state figure the
bench line's event-timed kernel_ms measures, from the same trace.

    python tools/steady_stats.py <kernel_trace.csv> <K> [out.json]

Same-named kernels launched in a fixed order per step (the multi-pass product's two k_cols8
passes) are told apart by their Kernel_Id order, as tools/summarize_profile.py does."""
import collections
import csv
import json
import statistics
import sys

path, k = sys.argv[1], int(sys.argv[2])
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ids = collections.defaultdict(set)
for r in rows:
    ids[r["Kernel_Name"]].add(int(r["Kernel_Id"]))
out = {}
for name in sorted(ids):
    short = name.split("(")[0].replace("void ", "").replace("nttmul::", "")
    kid = sorted(ids[name])
    for j, i in enumerate(kid):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
             if r["Kernel_Name"] == name and int(r["Kernel_Id"]) == i]
        key = short if len(kid) == 1 else f"{short}#{j}"
        tail = d[-k:]
        out[key] = {"dispatches": len(d), "mean_ms_all": statistics.mean(d),
                    "last_k": len(tail), "mean_ms_last_k": statistics.mean(tail),
                    "median_ms_last_k": statistics.median(tail),
                    "min_ms": min(d), "max_ms": max(d), "kernel": name[:160]}
res = {"trace": path, "k": k, "kernels": out}
if len(sys.argv) > 3:
    json.dump(res, open(sys.argv[3], "w"), indent=1)
print(json.dumps(res, indent=1))
