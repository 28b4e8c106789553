#!/bin/bash
# Round-5 re-check after host-only changes: the GPU parity suite, smoke() and the driver's exact
# bench command on the current tree.
set -o pipefail
OUT=gpurun_out/${1:-r5check}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_cmd.json 2> $OUT/driver_cmd.err || { tail -20 $OUT/driver_cmd.err; exit 1; }
tail -c 400 $OUT/driver_cmd.json
echo done
