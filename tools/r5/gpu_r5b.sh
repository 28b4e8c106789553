#!/bin/bash
# Round-5 GPU session B: GPU parity suite (tiled square split, server quiesce, N > 1 bench line),
# C5 A/B of the splits with disjoint-window store / load ablations (two interleaved rounds, board
# power per run), the energy microbenchmarks and the C3 kernel's pricing variants for the C3
# energy budget, then bench lines for C3 and C5 and a rocprofv3 kernel-stats pass of C5.
set -o pipefail
OUT=gpurun_out/r5b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.txt 2>&1
rc=$?; tail -5 $OUT/gpu_tests.txt
case $rc in 124|134|137|139) echo "tests died rc=$rc"; exit $rc;; esac
K=tools/kbench/bin; Q=4611686018425815041
for i in 1 2; do
  for v in t_base u_base o_base t_spec t_st t_ld t_ldst t_all o_st o_ld o_ldst o_all; do
    tools/power_trace.sh $OUT/c5ab$i $v $K/kbench_$v 65536 $Q 1024 3000 || exit 1
    cat $OUT/c5ab$i/$v.out
  done
done 2>&1 | tee $OUT/c5ab.txt
timeout -k 10 300 python tools/r5/energy_budget.py --seconds 3 > $OUT/energy.json 2> $OUT/energy.err || exit 1
cat $OUT/energy.err
for v in base noload nostore noxchg compute; do
  tools/power_trace.sh $OUT/c3abl $v $K/kbench_$v 4096 2013265921 65536 5000 || exit 1
  cat $OUT/c3abl/$v.out
done 2>&1 | tee $OUT/c3abl.txt
timeout -k 10 300 python bench.py > $OUT/c3_bench.json 2> $OUT/c3_bench.err || exit 1
timeout -k 10 300 python bench.py --n 65536 --q $Q --batch-per-gpu 1024 --steps 300 --warmup 20 \
  > $OUT/c5_bench.json 2> $OUT/c5_bench.err || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o c5 --output-format csv -- \
  python bench.py --n 65536 --q $Q --batch-per-gpu 1024 --steps 300 --warmup 20 --no-cpu-baseline \
  --power-seconds 0 --clock-seconds 0 > $OUT/prof_c5.log 2>&1 || exit 1
echo done
