#!/bin/bash
# C2 (n = 1024 x 4096, rotated over HBM) bench lines on 1..4 streams
set -o pipefail
mkdir -p gpurun_out/c2s
for s in ${STREAMS:-1 2 3 4}; do
  timeout -k 10 200 python bench.py --n 1024 --batch-per-gpu 4096 --steps 300 --warmup 50 --no-cpu-baseline --streams $s > gpurun_out/c2s/s$s.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/c2s/s$s.json').read().splitlines()[-1]); r=d['roofline']; print('C2 streams $s', round(d['value']/1e6,1), 'M/s', round(r['frac'],4), round(r['kernel_ms']*1e3,2), 'us', r['buffer_sets'], r['cache_resident'])"
done
