#!/bin/bash
# PMC comparison of kbench variants: VARIANTS="a b" ARGS="n q batch reps" tools/kbench/pmc_ab.sh
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B=tools/kbench/bin
OUT=gpurun_out/pmcab
mkdir -p $OUT
for v in $VARIANTS; do
  i=0
  SETS=${SETS:-"GRBM_GUI_ACTIVE,SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES;SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_WAIT_ANY;SQ_ACTIVE_INST_ANY,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INST_CYCLES_VMEM;SQ_ACTIVE_INST_LDS,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_MISC"}
  IFS=';' read -ra SETARR <<< "$SETS"
  for set0 in "${SETARR[@]}"; do
    set=${set0//,/ }
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -T --kernel-include-regex k_rows \
      -d $OUT/${v}_$i -o p --output-format csv -- $B/kbench_$v ${ARGS:-4096 2013265921 65536 3} > $OUT/${v}_$i.log 2>&1
  done
done
python3 - <<'PY'
import csv, glob, collections, os
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pmcab/*/p_counter_collection.csv'):
    v = os.path.basename(os.path.dirname(f)).rsplit('_', 1)[0]
    for r in csv.DictReader(open(f)):
        rows[v][r['Counter_Name']].append(float(r['Counter_Value']))
        rows[v]['dur_ns'].append(float(r['End_Timestamp']) - float(r['Start_Timestamp']))
for v, d in sorted(rows.items()):
    print(v)
    for k, xs in sorted(d.items()):
        print(f"  {k:24s} {sum(xs)/len(xs):16.1f}")
PY
