#!/bin/bash
# Round-5 session H: C2 with hardware kernel-argument preloading (kbench KB_PL: k_rows with a, b,
# c, units ahead of KParams, built with -amdgpu-kernarg-preload-count=8) against the base, three
# interleaved rounds over 16 rotated HBM buffer sets, 20,000 launches each.
set -o pipefail
OUT=gpurun_out/r5i; mkdir -p $OUT
export TMPDIR=/tmp
B=tools/kbench/bin
for i in 1 2 3; do
  for v in base pl; do
    echo -n "$v "; KB_ROTATE=16 timeout -k 5 60 $B/kbench_$v 1024 2013265921 4096 20000 || exit 1
  done
done 2>&1 | tee $OUT/pl.txt
echo done
