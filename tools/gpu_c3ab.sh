#!/bin/bash
# C3 kbench A/B (3 interleaved runs each): tools/gpu_c3ab.sh <tag> "<variants>"
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
VARIANTS="$2" timeout -k 10 500 tools/kbench/ab3.sh 4096 2013265921 65536 300 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
sort $OUT/ab.log | awk '{print $1, $6, $NF}'
