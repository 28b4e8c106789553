"""Summarise a tools/gpu_round.sh output directory into profiles/ (committed evidence).

    python tools/summarize_profile.py gpurun_out/<tag> profiles/<round>

Writes <round>_kernel_stats.csv (rocprofv3 --kernel-trace --stats of bench.py), <round>_pmc.json
(per-dispatch counter averages of the dominant kernel) and updates profiles/pmc_traffic.json, the
HBM-bytes-per-launch table bench.py reads for roofline.traffic.  FETCH_SIZE is doubled per
MI355X_MICROARCH.md §HBM (gfx950 reports half the bytes of coalesced streaming reads; checked on
this kernel: 2 x FETCH_SIZE = the 2 GiB of a and b it reads, within 0.05 %); WRITE_SIZE is exact.
"""
import csv
import collections
import json
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
shutil.copy(os.path.join(src, "trace", "trace_kernel_stats.csv"), dst + "_kernel_stats.csv")
bench = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
shutil.copy(os.path.join(src, "bench.json"), dst + "_bench.json")

pmc = collections.defaultdict(list)
dur = collections.defaultdict(list)
for root, _, files in os.walk(os.path.join(src, "pmc")):
    for f in files:
        if not f.endswith("_counter_collection.csv"):
            continue
        rows = sorted(csv.DictReader(open(os.path.join(root, f))), key=lambda r: int(r["Dispatch_Id"]))
        # kernels that share a truncated name (the square split's k_cols8 forward and inverse)
        # are told apart by their kernel id, numbered in order of first dispatch (the same order
        # in every pass: each pass runs the same program); the ids themselves differ per pass
        ids = collections.defaultdict(list)
        for r in rows:
            if r["Kernel_Id"] not in ids[r["Kernel_Name"]]:
                ids[r["Kernel_Name"]].append(r["Kernel_Id"])
        for r in rows:
            k = r["Kernel_Name"]
            if len(ids[k]) > 1:
                k = f"{k}#{ids[k].index(r['Kernel_Id'])}"
            pmc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = {}
for (k, c), v in sorted(pmc.items()):
    out.setdefault(k, {})[c] = sum(v) / len(v)
for k in out:
    out[k]["profiled_duration_ns_avg"] = sum(dur[k]) / len(dur[k])
json.dump(out, open(dst + "_pmc.json", "w"), indent=1)

cfg = bench["config"]
entry_co = bench.get("build", {}).get("code_object")
# the kernels one step dispatches, {kernel_key: hash of its machine code} (bench.py build.kernels):
# bench.py looks the entry up by these, kernel by kernel
entry_kernels = bench.get("build", {}).get("kernels")
if not entry_kernels:
    sys.exit("bench line without build.kernels (per-kernel hashes): profile a current bench.py")
main = "k_rows" if "k_rows" in out else sorted(out)[0]
m = out[main]
# one step = one dispatch of each product kernel (k_rows; plus k_cols_fwd/k_cols_inv for n > 4096)
step_kernels = sorted(k for k in out if k.startswith(("k_rows", "k_cols")))
fetch = sum(2.0 * out[k].get("FETCH_SIZE", 0.0) * 1024 for k in step_kernels)
write = sum(out[k].get("WRITE_SIZE", 0.0) * 1024 for k in step_kernels)
tpath = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
table = json.load(open(tpath)) if os.path.exists(tpath) else {"entries": []}
table["entries"] = [e for e in table["entries"]
                    if not (e["n"] == cfg["n"] and e["q"] == cfg["q"] and e["batch"] == cfg["batch_per_gpu"]
                            and e.get("kernels") == entry_kernels)]
entry = {"n": cfg["n"], "q": cfg["q"], "batch": cfg["batch_per_gpu"], "kernel": "+".join(step_kernels),
         "code_object": entry_co, "kernels": entry_kernels,
         "hbm_bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
         "alg_bytes_per_launch": bench["roofline"]["alg_bytes_per_launch"],
         "traffic_over_alg": (fetch + write) / bench["roofline"]["alg_bytes_per_launch"],
         "source": os.path.basename(dst) + "_pmc.json",
         "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                   "KB x 1024; FETCH_SIZE x 2 (gfx950 half-count of coalesced reads)"}
if "GRBM_GUI_ACTIVE" in m:
    entry["clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8 / m["profiled_duration_ns_avg"]
table["entries"].append(entry)
json.dump(table, open(tpath, "w"), indent=1)
print(json.dumps(entry, indent=1))
