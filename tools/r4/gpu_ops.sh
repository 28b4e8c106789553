# SURVEY 8(f) row 1 measured like the product: bench.py --op forward / inverse / pointwise at the
# C3 shape (and forward / inverse at C5's), each with a rocprofv3 kernel-stats pass.
set -o pipefail
T=${1:-r4ops}
OUT=gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --clock-seconds 0 "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), 'M', d['unit'], round(d['roofline']['kernel_ms'],4), 'ms', round(d['roofline']['frac'],3))" $OUT/$name.json $name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name.prof -o trace --output-format csv -- python3 bench.py --no-cpu-baseline --clock-seconds 0 --power-seconds 0 "$@" > $OUT/$name.prof.log 2>&1 || { tail -20 $OUT/$name.prof.log; exit 1; }
  cat $(find $OUT/$name.prof -name '*kernel_stats.csv' | head -1) | head -4
}
run c3_forward --op forward
run c3_inverse --op inverse
run c3_pointwise --op pointwise
run c5_forward --op forward --n 65536 --q 4611686018425815041 --batch-per-gpu 1024 --steps 200 --warmup 100
run c5_inverse --op inverse --n 65536 --q 4611686018425815041 --batch-per-gpu 1024 --steps 200 --warmup 100
