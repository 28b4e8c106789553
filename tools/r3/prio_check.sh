# Library build with the issue-prioritised k_rows variant: GPU parity suite, then kbench A/B of
# the automatic choice against forced off / on (NTTMUL_PRIO), and the C2 / C3 bench lines
set -o pipefail
OUT=gpurun_out/${1:-r3_prioc4}; mkdir -p $OUT
B=tools/kbench/bin
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
{
for i in 1 2; do for p in 0 auto; do echo -n "prio=$p "; NTTMUL_PRIO=${p/auto/} KB_ROTATE=16 timeout -k 5 60 $B/kbench_base 1024 2013265921 4096 2000 || exit 1; done; done
for p in 0 auto; do echo -n "prio=$p "; NTTMUL_PRIO=${p/auto/} timeout -k 5 60 $B/kbench_base 4096 2013265921 65536 100 || exit 1; done
for p in 0 auto; do echo -n "prio=$p "; NTTMUL_PRIO=${p/auto/} timeout -k 5 60 $B/kbench_base 1024 2013265921 262144 50 || exit 1; done
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
run() { local name=$1; shift; timeout -k 10 240 python bench.py --no-cpu-baseline --power-seconds 0 "$@" > $OUT/$name.json 2> $OUT/$name.err || exit 1
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step', d['roofline']['kernel'])"; }
run c2 --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000
run c3 --steps 100 --warmup 50
run c2s --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000 --streams 2
timeout -k 10 200 python -u tools/r3/c2_host_overhead.py > $OUT/host_overhead.txt 2>&1 || exit 1; tail -1 $OUT/host_overhead.txt
