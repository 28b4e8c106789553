# Standalone transforms after a change: their GPU tests, then the forward / inverse bench lines
set -o pipefail
T=${1:-r4x}
OUT=gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "transform or wrapper or cyclic" > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for op in forward inverse; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --clock-seconds 0 --op $op > $OUT/c3_$op.json 2> $OUT/c3_$op.err || { tail -20 $OUT/c3_$op.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M', d['unit'], round(d['roofline']['kernel_ms'],4), 'ms', round(d['roofline']['frac'],3))" $OUT/c3_$op.json $op
done
