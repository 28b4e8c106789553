#!/bin/bash
# C5 (n=65536, 62-bit q, batch 1024) A/B of kbench variants + per-kernel rocprof breakdown
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B=tools/kbench/bin
mkdir -p gpurun_out/c5
for i in 1 2; do for v in ${VARIANTS:-full full1}; do timeout -k 5 60 $B/kbench_$v 65536 4611686018425815041 1024 20; done; done > gpurun_out/c5/ab.txt 2>&1
cat gpurun_out/c5/ab.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5/prof -o c5 --output-format csv -- $B/kbench_${PROFV:-full} 65536 4611686018425815041 1024 20 > gpurun_out/c5/prof.log 2>&1
cat $(find gpurun_out/c5/prof -name "*kernel_stats.csv")
