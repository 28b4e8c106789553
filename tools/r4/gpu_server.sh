# Device-server checks: the server and shim GPU tests, the server's latency and timeline, and the
# relinked reference harness's per-call time (three runs).
set -o pipefail
T=${1:-r4h}
OUT=gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "server or shim or time_testing or kat or fpga" > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python tools/r4/server_latency.py > $OUT/server_latency.json 2> $OUT/server_latency.err || { tail -20 $OUT/server_latency.err; exit 1; }
grep -A3 '"server"' $OUT/server_latency.json; grep -A9 timeline $OUT/server_latency.json
A=ntt-based-polynomial-multiplier-fpga_amd/apps/time_testing_gpu
for i in 1 2 3; do
  timeout -k 10 120 $A tests/golden/coeficientes_a.txt tests/golden/coeficientes_b.txt 2000 > $OUT/time_testing_$i.txt 2>&1 || { tail -5 $OUT/time_testing_$i.txt; exit 1; }
  grep "us por" $OUT/time_testing_$i.txt
done
# one n = 1024 product (C1's shape) through the server, for the record
timeout -k 10 120 python tools/r4/server_latency.py --n 1024 --q 2013265921 > $OUT/server_latency_1024.json 2> $OUT/server_latency_1024.err || { tail -20 $OUT/server_latency_1024.err; exit 1; }
grep -A3 '"server"' $OUT/server_latency_1024.json; grep -A3 '"launch_per_call"' $OUT/server_latency_1024.json; grep compute_ns $OUT/server_latency_1024.json
# four n = 256 products per request (one pair of waves each)
timeout -k 10 120 python tools/r4/server_latency.py --batch 4 > $OUT/server_latency_b4.json 2> $OUT/server_latency_b4.err || { tail -20 $OUT/server_latency_b4.err; exit 1; }
grep -A3 '"server"' $OUT/server_latency_b4.json; grep compute_ns $OUT/server_latency_b4.json
