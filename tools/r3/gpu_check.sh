# Round-3 GPU check: parity tests, smoke, the default bench line, C5/C2 lines, counter list.
set -o pipefail
OUT=gpurun_out/${1:-r3a}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/c3_bench.json 2> $OUT/c3_bench.err || { tail -20 $OUT/c3_bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c3_bench.json'));print('C3',d['value']/1e6,d['roofline']['frac'],d['roofline']['kernel'],d['cpu_baseline'].get('c1'),d['cpu_baseline'].get('host_cores'))"
timeout -k 10 300 python bench.py --n 65536 --q 4611686018425815041 --batch-per-gpu 1024 --no-cpu-baseline --power-seconds 0 > $OUT/c5_bench.json 2> $OUT/c5_bench.err || { tail -20 $OUT/c5_bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c5_bench.json'));print('C5',d['value']/1e6,d['roofline']['frac'],d['roofline']['kernel'])"
timeout -k 10 300 python bench.py --n 1024 --batch-per-gpu 4096 --steps 2000 --warmup 200 --no-cpu-baseline --power-seconds 0 > $OUT/c2_bench.json 2> $OUT/c2_bench.err || { tail -20 $OUT/c2_bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/c2_bench.json'));print('C2',d['value']/1e6,d['roofline']['frac'],d['roofline']['kernel'])"
timeout -k 10 120 rocprofv3 --list-avail > $OUT/counters.txt 2>&1 || true
grep -i -E "mall|dram|EA0_RD|EA0_WR|TCC_EA" $OUT/counters.txt | head -40
