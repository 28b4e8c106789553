#!/bin/bash
# Round-5 evidence for the build, in two calls (each under gpurun's 20-minute limit):
#   part 1: GPU parity suite + smoke, bench lines + rocprofv3 kernel stats + PMC traffic passes
#           for C3 and C5 (tools/gpu_prof.sh)
#   part 2: the same for C2 (+ two streams), SURVEY 8(f) row 1's standalone transforms / pointwise
#           (tools/r4/gpu_ops.sh), the driver's exact bench command, and the relinked reference
#           harness against the reference's CPU code on this host (tools/r5/server_vs_ref.py)
# usage: tools/r5/gpu_final.sh <tag> <1|2>
set -o pipefail
TAG=${1:-r5final}; PART=${2:-1}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ "$PART" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
  bash tools/gpu_prof.sh $TAG c3 c5 2> $OUT/prof.log || { tail -30 $OUT/prof.log; exit 1; }
  tail -5 $OUT/prof.log
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "multipass_vs_oracle or small_server" > $OUT/gpu_tests2.log 2>&1 || { tail -60 $OUT/gpu_tests2.log; exit 1; }
  tail -1 $OUT/gpu_tests2.log
  bash tools/gpu_prof.sh $TAG c2 c2s 2> $OUT/prof2.log || { tail -30 $OUT/prof2.log; exit 1; }
  tail -5 $OUT/prof2.log
  bash tools/r4/gpu_ops.sh $TAG/ops > $OUT/ops.log 2>&1 || { tail -20 $OUT/ops.log; exit 1; }
  grep " M " $OUT/ops.log
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_cmd.json 2> $OUT/driver_cmd.err || { tail -20 $OUT/driver_cmd.err; exit 1; }
  tail -c 600 $OUT/driver_cmd.json
  timeout -k 10 300 python3 tools/r5/server_vs_ref.py > $OUT/server_vs_ref.json 2> $OUT/server_vs_ref.err || { tail -20 $OUT/server_vs_ref.err; exit 1; }
  cat $OUT/server_vs_ref.json
fi
echo "done $TAG part $PART"
