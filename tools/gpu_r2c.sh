#!/bin/bash
# Round-2 session C: Plantard vs Montgomery kbench A/B (C3, C2-shape, C5), GPU parity tests,
# C3 bench line.  Usage: tools/gpu_r2c.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r2c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, timeout, command...: stop the session at the first failure
  local name=$1 t=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED $name rc=$rc" >&2; tail -40 $OUT/$name.log >&2; exit $rc; fi
  tail -4 $OUT/$name.log >&2
}
export VARIANTS="base prev nofold notyped lds1 compute"; step ab_c3 300 tools/kbench/ab3.sh 4096 2013265921 65536 100
export VARIANTS="base prev"; step ab_n1024 200 tools/kbench/ab3.sh 1024 2013265921 262144 100
if [ "$2" != "skip-tests" ]; then
  step gpu_tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
fi
step bench 300 python bench.py
echo "done $TAG" >&2
