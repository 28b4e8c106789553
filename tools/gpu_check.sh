#!/bin/bash
# GPU parity tests + smoke + C3 bench of the current tree: tools/gpu_check.sh <tag>
set -o pipefail
if [ "$1" = "--help" ]; then sed -n 2p "$0"; exit 0; fi
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/gpu_tests.log | tail -20; tail -60 $OUT/gpu_tests.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); print('C3', round(d['value']/1e6,2), 'M/s', round(d['roofline']['frac'],4), d['roofline']['kernel_ms'], d['build']['kernels'])"
