#!/bin/bash
# Round-2 GPU session: parity tests, the C3 bench line, rocprofv3 kernel stats, and the C2/C5
# sweeps (Infinity-Cache rotation; multi-pass sub-batch size).  Usage: tools/gpu_r2.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, timeout, command...: stop the session at the first failure
  local name=$1 t=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED $name rc=$rc" >&2; tail -40 $OUT/$name.log >&2; exit $rc; fi
  tail -3 $OUT/$name.log >&2
}
if [ "$2" != "skip-tests" ]; then
  step gpu_tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
fi
step bench 300 python bench.py
cp $OUT/bench.log $OUT/bench.json
step trace 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o trace --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 200 --warmup 20
for mb in 8 16 32 64 128; do
  NTTMUL_MP_CHUNK_MB=$mb step c5_mb$mb 300 python bench.py --n 65536 --q 4611686018425815041 \
    --batch-per-gpu 1024 --steps 30 --warmup 10 --no-cpu-baseline
done
step c2_rot 300 python bench.py --n 1024 --batch-per-gpu 4096 --steps 200 --warmup 50 --no-cpu-baseline
step c2_norot 300 python bench.py --n 1024 --batch-per-gpu 4096 --steps 200 --warmup 50 --no-cpu-baseline --rotate 1
echo "done $TAG" >&2
