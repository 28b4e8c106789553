# Kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the runtime default, interleaved:
# does the first scalar load of each launch wait on host memory?  C2 (one stream) and C3 lines.
set -o pipefail
OUT=gpurun_out/${1:-r3_kernarg}; mkdir -p $OUT
: > $OUT/out.txt
c2="--n 1024 --batch-per-gpu 4096 --steps 3000 --warmup 2000"
for i in 1 2; do for v in default 1 0; do
  if [ $v = default ]; then E=""; else E="HIP_FORCE_DEV_KERNARG=$v"; fi
  env $E timeout -k 10 120 python bench.py $c2 --no-cpu-baseline --power-seconds 0 > $OUT/l.json 2>> $OUT/err.txt || exit 1
  python -c "import json; d=json.loads(open('$OUT/l.json').read()); print('C2 kernarg=$v', round(d['value']/1e6,2), 'M/s kernel_us', round(d['roofline']['kernel_ms']*1e3,3))" >> $OUT/out.txt
done; done
for v in default 1 0; do
  if [ $v = default ]; then E=""; else E="HIP_FORCE_DEV_KERNARG=$v"; fi
  env $E timeout -k 10 120 python bench.py --no-cpu-baseline --power-seconds 0 > $OUT/l.json 2>> $OUT/err.txt || exit 1
  python -c "import json; d=json.loads(open('$OUT/l.json').read()); print('C3 kernarg=$v', round(d['value']/1e6,2), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4))" >> $OUT/out.txt
done
cat $OUT/out.txt
