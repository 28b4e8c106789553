#!/bin/bash
# Ablation timings + sustained clock (GRBM_GUI_ACTIVE per XCD / kernel duration) per variant
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B=tools/kbench/bin
OUT=gpurun_out/ablclk
mkdir -p $OUT
for i in 1 2; do for v in ${VARIANTS:-base noload noxchg nostore compute}; do timeout -k 5 60 $B/kbench_$v ${ARGS:-4096 2013265921 65536 100}; done; done > $OUT/times.txt 2>&1
for v in ${VARIANTS:-base noload noxchg nostore compute}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES -T --kernel-include-regex k_rows \
    -d $OUT/$v -o p --output-format csv -- $B/kbench_$v ${ARGS:-4096 2013265921 65536 30} > $OUT/$v.log 2>&1
done
python3 - <<'PY'
import csv, glob, collections, os
for f in sorted(glob.glob('gpurun_out/ablclk/*/p_counter_collection.csv')):
    v = os.path.basename(os.path.dirname(f))
    d = collections.defaultdict(list); dur = []
    for r in csv.DictReader(open(f)):
        d[r['Counter_Name']].append(float(r['Counter_Value']))
        dur.append(float(r['End_Timestamp']) - float(r['Start_Timestamp']))
    g = sum(d['GRBM_GUI_ACTIVE'])/len(d['GRBM_GUI_ACTIVE']) / 8
    t = sum(dur)/len(dur)
    print(f"{v:10s} dur {t/1e6:.3f} ms  cycles/XCD {g/1e6:.3f} M  clock {g/t:.3f} GHz  valu/wave {sum(d['SQ_INSTS_VALU'])/sum(d['SQ_WAVES']):.0f}")
PY
cat $OUT/times.txt
