#!/bin/bash
# Evidence session for the current build (GPU box, repo root): the GPU parity suite and smoke(),
# the driver's own bench command (C3), and bench lines for C5, C2 and C2 on two streams, each step
# under its own time limit; then, with LIB set, same-box A/B bench lines of this build against
# another libnttmul.so (tools/bench_ab.py, interleaved, two rounds) at C3 and C5.
#   tools/gpu_evidence.sh <tag>            LIB=<other libnttmul.so> tools/gpu_evidence.sh <tag>
set -o pipefail
if [ "$1" = "--help" ] || [ -z "$1" ]; then sed -n 2,6p "$0"; exit 0; fi
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
Q5=4611686018425815041
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.txt 2>&1 || { grep -E "FAILED|Error" $OUT/gpu_tests.txt | tail; tail -40 $OUT/gpu_tests.txt; exit 1; }
tail -1 $OUT/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
line() {  # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().splitlines()[-1]); r=d['roofline']; print('$name', round(d['value']/1e6,4), 'M/s', round(r['frac'],4), round(r['kernel_ms'],5), 'traffic', r['traffic'] is not None, 'valu', 'valu_roofline' in d)"
}
line c3_driver_cmd 300 --gpus 1 --steps 20 --warmup 5
line c5 300 --n 65536 --q $Q5 --batch-per-gpu 1024 --steps 200 --warmup 100
line c2 300 --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000
line c2s 300 --n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000 --streams 2 --no-cpu-baseline
if [ -n "$LIB" ]; then
  for i in 1 2; do
    for side in new old; do
      L=ntt-based-polynomial-multiplier-fpga_amd/lib/libnttmul.so; [ $side = old ] && L=$LIB
      for cfg in c3 c5; do
        A=""; [ $cfg = c5 ] && A="--n 65536 --q $Q5 --batch-per-gpu 1024 --steps 200 --warmup 100"
        timeout -k 10 300 python3 tools/bench_ab.py $L $A > $OUT/ab_${cfg}_${side}_$i.json 2> $OUT/ab_${cfg}_${side}_$i.err || { tail -20 $OUT/ab_${cfg}_${side}_$i.err; exit 1; }
        python3 -c "import json; d=json.loads(open('$OUT/ab_${cfg}_${side}_$i.json').read().splitlines()[-1]); print('ab $cfg $side $i', round(d['value']/1e6,4), round(d['roofline']['kernel_ms'],5), d['power'].get('socket_power_w_median'), d['ab_library']['code_object'])"
      done
    done
  done
fi
echo "done $1"
