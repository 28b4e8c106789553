#!/bin/bash
# Evidence session for the current build: bench lines + rocprofv3 kernel stats + PMC traffic
# passes for C3 (bench default), C5 and C2, each step under its own time limit.
# Usage (GPU box, repo root): tools/gpu_prof.sh <tag> [cfg...]; then locally
#   python tools/summarize_profile.py gpurun_out/<tag>/<cfg> profiles/r2/<cfg>
set -o pipefail
TAG=${1:-prof}
shift
CFGS=${@:-c3 c5 c2}
export TMPDIR=/tmp
run() {  # timeout, command...
  local t=$1; shift
  timeout -k 10 $t "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED ($rc): $*" >&2; exit $rc; fi
}
one() {  # cfg name, bench args...
  local cfg=$1; shift
  local OUT=gpurun_out/$TAG/$cfg
  mkdir -p $OUT
  echo "== $cfg" >&2
  run 300 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
  tail -c 700 $OUT/bench.json >&2
  run 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o trace --output-format csv -- \
    python3 bench.py --no-cpu-baseline --power-seconds 0 --clock-seconds 0 "$@" > $OUT/trace.log 2>&1
  run 900 tools/profile_pmc.sh $OUT/pmc "$@" --no-cpu-baseline --power-seconds 0 --clock-seconds 0 --settle-ms 0 --steps 3 --warmup 1 > $OUT/pmc.log 2>&1
}
for cfg in $CFGS; do
  case $cfg in
    c3) one c3 ;;
    c5) one c5 --n 65536 --q 4611686018425815041 --batch-per-gpu 1024 --steps 200 --warmup 100 ;;
    c2) one c2 --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000 ;;
    c2s) one c2s --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000 --streams 2 ;;  # two streams: the oldest-first kernel
  esac
done
echo "done $TAG" >&2
