#!/bin/bash
# Power / clock evidence session: board power and shader clock while C3 (bench), the kbench base /
# no-load / compute-only ablations and C5 run (tools/power_trace.sh; read-only amd-smi queries).
set -o pipefail
OUT=gpurun_out/power
mkdir -p $OUT
timeout -k 5 30 amd-smi static -g 0 --json > $OUT/static.json 2>&1
timeout -k 5 30 amd-smi metric -g 0 --json > $OUT/idle.json 2>&1
T=tools/power_trace.sh
$T $OUT c3_bench python bench.py --steps 10000 --warmup 50 --no-cpu-baseline || exit 1
K=tools/kbench/bin
for v in base noload compute; do
  $T $OUT kb_$v $K/kbench_$v 4096 2013265921 65536 10000 || exit 1
done
$T $OUT c5_bench python bench.py --n 65536 --q 4611686018425815041 --batch-per-gpu 1024 --steps 6000 --warmup 10 --no-cpu-baseline || exit 1
echo done
