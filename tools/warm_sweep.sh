set -e
mkdir -p gpurun_out/warm
for cfg in "5 20" "50 100" "200 20" "20 500"; do set -- $cfg; timeout -k 10 120 python bench.py --no-cpu-baseline --warmup $1 --steps $2 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('W=$1 K=$2', round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4))"; done > gpurun_out/warm/out.txt 2>&1
cat gpurun_out/warm/out.txt
