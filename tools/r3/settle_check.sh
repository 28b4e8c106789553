# The driver's exact bench command after the settle phase (bench.py --settle-ms, default 200),
# twice, beside --settle-ms 0; then the 2-rank bench test (bench.py changed).
set -o pipefail
OUT=gpurun_out/${1:-r3_settle}; mkdir -p $OUT
: > $OUT/out.txt
for s in 200 0 200; do
  timeout -k 10 180 python3 bench.py --gpus 1 --steps 20 --warmup 5 --settle-ms $s > $OUT/line_$s.json 2>> $OUT/err.txt || exit 1
  python -c "import json; d=json.loads(open('$OUT/line_$s.json').read()); print('settle=$s', d.get('settle'), round(d['value']/1e6,2), 'M/s kernel_ms', round(d['roofline']['kernel_ms'],4), 'power', d.get('power',{}).get('socket_power_w_median'))" >> $OUT/out.txt
done
cat $OUT/out.txt
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "bench_two_ranks or smoke or full_size_device_path" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
