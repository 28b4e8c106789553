#!/bin/bash
# Bench line + rocprofv3 kernel stats for the parity configurations C2 and C5 (the bench's own
# line is C3).  Usage on the GPU box, from the repo root: tools/configs_prof.sh <outdir>
set -e
OUT=${1:-gpurun_out/cfg}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/${name}_bench.json 2> $OUT/${name}_bench.err
  tail -1 $OUT/${name}_bench.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/$name -o $name --output-format csv -- \
    python3 bench.py --no-cpu-baseline "$@" > $OUT/${name}_trace.log 2>&1
}
run c2 --n 1024 --batch-per-gpu 4096 --steps 200 --warmup 50
run c5 --n 65536 --q 4611686018425815041 --batch-per-gpu 1024 --steps 50 --warmup 10
echo "configs done"
