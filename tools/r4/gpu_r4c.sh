# Round-4 second GPU session: the GPU parity suite on the rebuilt library (Arith64 CT sum from the
# Shoup addend), the device server's latency and timeline, the C5 sub-batch pipeline A/B, the
# C5 Infinity-Cache ablations, and the random-operand multiply energies.
set -o pipefail
T=${1:-r4c}
OUT=gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python tools/r4/server_latency.py > $OUT/server_latency.json 2> $OUT/server_latency.err || { tail -20 $OUT/server_latency.err; exit 1; }
cat $OUT/server_latency.json
bash tools/r4/c5_pipe_ab.sh ${T}_c5pipe > /dev/null || exit 1
grep -h "==\|Mpolymul" gpurun_out/${T}_c5pipe/ab.txt | paste - - | awk '{print $2, $8, $9, $NF}'
bash tools/r4/c5_ic_ablation.sh ${T}_c5ic > /dev/null || exit 1
awk '{print $1, $6, $7, $NF}' gpurun_out/${T}_c5ic/ab.txt
timeout -k 10 240 python tools/r4/valu_energy.py --seconds 3 --kinds 0,9,10,1,2,14,15,16,3 > $OUT/valu_energy.json 2> $OUT/valu_energy.err || { tail -30 $OUT/valu_energy.err; exit 1; }
cat $OUT/valu_energy.err
