# Round-4 evidence for the final build, part 2: C2 (one and two streams) and the C4 per-rank
# slice with rocprofv3 / PMC (tools/gpu_prof.sh), the relinked reference harness's per-call
# time, and the device server's latency and timeline.
set -o pipefail
TAG=${1:-r4final}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_prof.sh $TAG c2 c2s 2> $OUT/prof2.log || { tail -30 $OUT/prof2.log; exit 1; }
tail -3 $OUT/prof2.log
timeout -k 10 300 python bench.py --batch-per-gpu 131072 --no-cpu-baseline > $OUT/c4slice_bench.json 2> $OUT/c4slice_bench.err || { tail -20 $OUT/c4slice_bench.err; exit 1; }
tail -c 300 $OUT/c4slice_bench.json
A=ntt-based-polynomial-multiplier-fpga_amd/apps/time_testing_gpu
for i in 1 2 3; do
  timeout -k 10 120 $A tests/golden/coeficientes_a.txt tests/golden/coeficientes_b.txt 2000 > $OUT/time_testing_$i.txt 2>&1 || { tail -5 $OUT/time_testing_$i.txt; exit 1; }
  grep "us por" $OUT/time_testing_$i.txt
done
timeout -k 10 120 python tools/r4/server_latency.py > $OUT/server_latency.json 2> $OUT/server_latency.err || { tail -20 $OUT/server_latency.err; exit 1; }
grep -A8 timeline $OUT/server_latency.json
# the reference's own ntt256_product4 etc. on one core of this box (oracle/_ref, checked against
# the oracle), beside the server's per-call time above
timeout -k 10 120 python -c "import json, sys; sys.path.insert(0, '.'); from oracle import oracle as O; print(json.dumps({k: v * 1e6 for k, v in O.ref_anchors().items()}, indent=1))" > $OUT/ref_anchors_us.json || exit 1
cat $OUT/ref_anchors_us.json
