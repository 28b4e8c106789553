#!/bin/bash
# Round-5 GPU session A: the GPU parity suite on the square-split C5 build, then C5 kbench A/B of
# the two splits with the intermediate store / load ablations (interleaved, two rounds, board
# power sampled per run), rocprofv3 kernel stats of both splits, and bench lines for C5 and C3.
set -o pipefail
OUT=gpurun_out/r5a; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.txt 2>&1
rc=$?; tail -5 $OUT/gpu_tests.txt
case $rc in 124|134|137|139) echo "tests died rc=$rc"; exit $rc;; esac
K=tools/kbench/bin; Q=4611686018425815041
for i in 1 2; do
  for v in o_base n_base o_st n_st o_ld n_ld o_ldst n_ldst o_all n_all n_basepl n_stpl; do
    tools/power_trace.sh $OUT/ab$i $v $K/kbench_$v 65536 $Q 1024 3000 || exit 1
    cat $OUT/ab$i/$v.out
  done
done 2>&1 | tee $OUT/ab.txt
for v in o_base n_base; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run -- $K/kbench_$v 65536 $Q 1024 300 \
    > $OUT/prof_$v.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --n 65536 --q $Q --batch-per-gpu 1024 --steps 300 --warmup 20 \
  > $OUT/c5_bench.json 2> $OUT/c5_bench.err || exit 1
timeout -k 10 300 python bench.py > $OUT/c3_bench.json 2> $OUT/c3_bench.err || exit 1
echo done
