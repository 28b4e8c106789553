# C2 / C5 bench lines at the default short runs vs longer warmups (clock ramp), one box
set -o pipefail
OUT=gpurun_out/${1:-r3_steps}; mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 240 python bench.py --no-cpu-baseline --power-seconds 0 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step', 'kernel', round(d['roofline']['kernel_ms']*1e3,2))"; }
run c2_300_50 --n 1024 --batch-per-gpu 4096 --steps 300 --warmup 50
run c2_3000_2000 --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000
run c2_300_50b --n 1024 --batch-per-gpu 4096 --steps 300 --warmup 50
run c2_3000_2000b --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000
run c2s_3000_2000 --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000 --streams 2
run c5_30_10 --n 65536 --q 4611686018425815041 --batch-per-gpu 1024 --steps 30 --warmup 10
run c5_200_100 --n 65536 --q 4611686018425815041 --batch-per-gpu 1024 --steps 200 --warmup 100
run c3_100_50 --steps 100 --warmup 50
run c3_500_300 --steps 500 --warmup 300
