#!/bin/bash
# C5 pipelined multi-pass sweep: lanes x sub-batch size (bench.py, one process per point)
set -o pipefail
OUT=gpurun_out/${1:-c5sweep}
mkdir -p $OUT
for lanes in 1 2; do
  for mb in ${MBS:-16 32 64 128 256 512}; do
    NTTMUL_MP_LANES=$lanes NTTMUL_MP_CHUNK_MB=$mb timeout -k 10 120 python bench.py --n 65536 \
      --q 4611686018425815041 --batch-per-gpu 1024 --steps 30 --warmup 10 --no-cpu-baseline \
      > $OUT/l${lanes}_mb$mb.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('$OUT/l${lanes}_mb$mb.json').read().splitlines()[-1]); print('lanes $lanes mb $mb', round(d['roofline']['kernel_ms'],4), 'ms', round(d['value']/1e6,3), 'M/s')"
  done
done | tee $OUT/summary.txt
