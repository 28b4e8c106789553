#!/bin/bash
# kbench A/B session: tools/gpu_ab.sh <tag> "<variants>" "<kbench args>" ["<variants>" "<args>" ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
while [ $# -ge 2 ]; do
  i=$((i+1))
  export VARIANTS="$1"
  echo "== $VARIANTS :: $2" | tee -a $OUT/ab.txt
  timeout -k 10 400 tools/kbench/ab3.sh $2 > $OUT/ab_$i.log 2>&1 || { echo "FAILED ab $i"; cat $OUT/ab_$i.log; exit 1; }
  sort $OUT/ab_$i.log | awk '{print $1, $6}' | tee -a $OUT/ab.txt
  shift 2
done
