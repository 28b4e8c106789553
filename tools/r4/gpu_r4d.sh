# Device server with wide staged loads/stores and lane-split transforms: GPU suite, server
# latency + timeline, the relinked reference harness's per-call time.
set -o pipefail
T=${1:-r4d}
OUT=gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python tools/r4/server_latency.py > $OUT/server_latency.json 2> $OUT/server_latency.err || { tail -20 $OUT/server_latency.err; exit 1; }
cat $OUT/server_latency.json
A=ntt-based-polynomial-multiplier-fpga_amd/apps/time_testing_gpu
for i in 1 2 3; do
  timeout -k 10 120 $A tests/golden/coeficientes_a.txt tests/golden/coeficientes_b.txt 2000 > $OUT/time_testing_$i.txt 2>&1 || { tail -5 $OUT/time_testing_$i.txt; exit 1; }
  grep "Tempo\|us por" $OUT/time_testing_$i.txt
done
