#!/bin/bash
# Bench lines of the current build after its PMC/VALU profiles are recorded (traffic populated)
set -o pipefail
OUT=gpurun_out/r2z_b; mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/c3_bench.json 2> $OUT/c3.err || exit 1
timeout -k 10 300 python bench.py --n 65536 --q 4611686018425815041 --batch-per-gpu 1024 --steps 30 --warmup 10 --no-cpu-baseline > $OUT/c5_bench.json 2> $OUT/c5.err || exit 1
timeout -k 10 300 python bench.py --n 1024 --batch-per-gpu 4096 --steps 300 --warmup 50 --no-cpu-baseline > $OUT/c2_bench.json 2> $OUT/c2.err || exit 1
for c in c3 c5 c2; do tail -c 300 $OUT/${c}_bench.json; echo; done
