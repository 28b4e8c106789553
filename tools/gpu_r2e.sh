#!/bin/bash
# A/B of a kernel change + GPU parity tests + C3 bench: tools/gpu_r2e.sh <tag> "<variants>"
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
tools/gpu_ab.sh $TAG "$2" "4096 2013265921 65536 100" "$2" "1024 2013265921 4096 1000" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || { tail -60 $OUT/gpu_tests.log; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); print('C3', round(d['value']/1e6,2), 'M/s', round(d['roofline']['frac'],4), d['roofline']['kernel_ms'])"
