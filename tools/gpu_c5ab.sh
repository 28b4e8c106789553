#!/bin/bash
# C5 kbench A/B (3 interleaved runs each): tools/gpu_c5ab.sh <tag> "<variants>"
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
VARIANTS="$2" timeout -k 10 300 tools/kbench/ab3.sh 65536 4611686018425815041 1024 100 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
sort $OUT/ab.log
