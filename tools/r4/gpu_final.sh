# Round-4 evidence for the final build, part 1: GPU parity tests, smoke, then bench lines +
# rocprofv3 kernel stats + PMC passes (tools/gpu_prof.sh) for C3 and C5, and the driver's exact
# bench command.  Part 2: tools/r4/gpu_final2.sh.
set -o pipefail
TAG=${1:-r4final}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/gpu_prof.sh $TAG c3 c5 2> $OUT/prof.log || { tail -30 $OUT/prof.log; exit 1; }
tail -5 $OUT/prof.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_cmd.json 2> $OUT/driver_cmd.err || { tail -20 $OUT/driver_cmd.err; exit 1; }
tail -c 600 $OUT/driver_cmd.json
