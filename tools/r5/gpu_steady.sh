#!/bin/bash
# Round-5 session J: rocprofv3 kernel traces of the C3, C2 and C5 bench commands, reduced on the
# box to per-kernel means over the whole run and over the timed steps only (the last K dispatches;
# tools/r5/steady_stats.py), so the profile's steady-state launch time can be set beside the bench
# line's event-timed kernel_ms (rocprofv3 --stats averages the settle and clock-ramp launches in).
set -o pipefail
OUT=gpurun_out/r5j; mkdir -p $OUT
export TMPDIR=/tmp
prof() {  # name, K, bench args...
  local name=$1 k=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name -o $name --output-format csv -- \
    python3 bench.py --no-cpu-baseline --power-seconds 0 --clock-seconds 0 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
  tail -c 300 $OUT/$name.json
  python3 tools/r5/steady_stats.py $OUT/$name/${name}_kernel_trace.csv $k $OUT/${name}_steady.json > /dev/null || exit 1
  rm -f $OUT/$name/${name}_kernel_trace.csv
}
prof c3 100
prof c2 3000 --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000
prof c5 200 --n 65536 --q 4611686018425815041 --batch-per-gpu 1024 --steps 200 --warmup 100
echo done
