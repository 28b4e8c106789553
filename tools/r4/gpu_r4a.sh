# Round-4 first GPU session: per-instruction energy at the cap, the GPU parity suite on this
# round's library (knobs in nttmul_params, no persistent path), smoke, and the C3 bench with the
# in-kernel clock from lib/libnttmul_diag.so.
set -o pipefail
OUT=gpurun_out/${1:-r4a}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python tools/r4/valu_energy.py --seconds 3 > $OUT/valu_energy.json 2> $OUT/valu_energy.err || { tail -30 $OUT/valu_energy.err; exit 1; }
cat $OUT/valu_energy.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/c3_bench.json 2> $OUT/c3_bench.err || { tail -20 $OUT/c3_bench.err; exit 1; }
tail -c 1500 $OUT/c3_bench.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_cmd.json 2> $OUT/driver_cmd.err || { tail -20 $OUT/driver_cmd.err; exit 1; }
tail -c 300 $OUT/driver_cmd.json
