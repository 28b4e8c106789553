#!/bin/bash
# GPU tests, C5 pipelined-lanes A/B (interleaved), ntt256_product4 per-call latency.
set -o pipefail
OUT=gpurun_out/r2b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
C5="--n 65536 --q 4611686018425815041 --batch-per-gpu 1024 --steps 40 --warmup 10 --no-cpu-baseline"
for r in 1 2 3; do
  for cfg in "1 512" "2 64" "2 128"; do
    set -- $cfg
    NTTMUL_MP_LANES=$1 NTTMUL_MP_CHUNK_MB=$2 timeout -k 10 120 python bench.py $C5 > $OUT/c5_l$1_mb$2_$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/c5_l$1_mb$2_$r.json').read().splitlines()[-1]); print('lanes $1 mb $2 run $r', round(d['roofline']['kernel_ms'],4), 'ms')"
  done
done | tee $OUT/c5_ab.txt
APP=ntt-based-polynomial-multiplier-fpga_amd/apps/time_testing_gpu
G=tests/golden
timeout -k 10 120 $APP $G/coeficientes_a.txt $G/coeficientes_b.txt 2000 1 > $OUT/product4_latency.txt 2>&1 || exit 1
grep -i "tempo\|batch" $OUT/product4_latency.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -T -d $OUT/p4trace -o p4 --output-format csv -- $APP $G/coeficientes_a.txt $G/coeficientes_b.txt 2000 1 > $OUT/p4trace.log 2>&1 || exit 1
cat $OUT/p4trace/p4_kernel_stats.csv
