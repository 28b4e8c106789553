#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel-trace stats and PMC traffic passes.
# Usage (from the repo root on the box): tools/gpu_round.sh <tag>
set -e
TAG=${1:-r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o trace --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 200 --warmup 20 > $OUT/trace.log 2>&1
timeout -k 10 600 tools/profile_pmc.sh $OUT/pmc > $OUT/pmc.log 2>&1
echo "done $TAG"
