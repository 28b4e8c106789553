# GPU parity suite + smoke on this round's library, the relinked reference harness's per-call
# latency (ntt256_product4 through the device server), and the C3 bench with the in-kernel clock.
set -o pipefail
OUT=gpurun_out/${1:-r4b}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
A=ntt-based-polynomial-multiplier-fpga_amd/apps/time_testing_gpu
for i in 1 2 3; do
  timeout -k 10 120 $A tests/golden/coeficientes_a.txt tests/golden/coeficientes_b.txt 2000 > $OUT/time_testing_$i.txt 2>&1 || { tail -5 $OUT/time_testing_$i.txt; exit 1; }
  grep "Tempo" $OUT/time_testing_$i.txt
done
timeout -k 10 300 python bench.py > $OUT/c3_bench.json 2> $OUT/c3_bench.err || { tail -20 $OUT/c3_bench.err; exit 1; }
tail -c 1800 $OUT/c3_bench.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_cmd.json 2> $OUT/driver_cmd.err || { tail -20 $OUT/driver_cmd.err; exit 1; }
tail -c 300 $OUT/driver_cmd.json
bash tools/r4/c5_l2_ablation.sh ${1:-r4b}_c5l2 > /dev/null || exit 1
cat gpurun_out/${1:-r4b}_c5l2/ab.txt
