# two-stream C2 bench line: automatic issue priority (alternating streams -> off) vs forced off / on
set -o pipefail
OUT=gpurun_out/${1:-r3_c2sp}; mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 240 python bench.py --no-cpu-baseline --power-seconds 0 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step')"; }
for i in 1 2; do
  NTTMUL_PRIO= run c2s_auto --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000 --streams 2
  NTTMUL_PRIO=0 run c2s_off --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000 --streams 2
  NTTMUL_PRIO=1 run c2s_on --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000 --streams 2
  NTTMUL_PRIO= run c2_auto --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000
  NTTMUL_PRIO=0 run c2_off --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000
done
