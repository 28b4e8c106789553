# C2: does the one-stream rate keep rising with longer warmups (clock ramp), one box
set -o pipefail
OUT=gpurun_out/${1:-r3_long}; mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 240 python bench.py --no-cpu-baseline --power-seconds 0 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step', 'kernel', round(d['roofline']['kernel_ms']*1e3,2))"; }
run c2_3000_2000 --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000
run c2_10000_20000 --n 1024 --batch-per-gpu 4096 --steps 10000 --warmup 20000
run c2_3000_2000_p1 --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000 --power-seconds 1
run c2_10000_20000b --n 1024 --batch-per-gpu 4096 --steps 10000 --warmup 20000
