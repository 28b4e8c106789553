# C3 bench at the driver's --warmup 5 --steps 20 against the defaults, on one box: is the
# round-end number (BENCH_r02: 60.9 M/s, kernel 1.074 ms) the box or the short warm-up?
set -o pipefail
OUT=gpurun_out/${1:-r3_warm}; mkdir -p $OUT
: > $OUT/out.txt
for cfg in "5 20" "5 20" "50 100" "5 20" "200 20" "0 20" "5 20"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --no-cpu-baseline --power-seconds 0 --warmup $1 --steps $2 > $OUT/line.json 2>> $OUT/err.txt || exit 1
  python -c "import json; d=json.loads(open('$OUT/line.json').read()); print('W=$1 K=$2', round(d['value']/1e6,2), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4), 'ms_per_step', round(d['ms_per_step'],4))" >> $OUT/out.txt
  sleep 2
done
cat $OUT/out.txt
