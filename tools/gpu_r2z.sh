#!/bin/bash
# Parity tests, smoke, then the evidence session (tools/gpu_prof.sh) for the current build
set -o pipefail
OUT=gpurun_out/r2z; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
bash tools/gpu_prof.sh r2z c3 c5 c2
