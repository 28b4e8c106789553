# Re-key the committed profiles to the final code object: full GPU suite + smoke, C3 / C5 / C2
# bench lines with rocprof stats and PMC passes, the driver's command, server + anchors.
set -o pipefail
T=${1:-r4final4}
bash tools/r4/gpu_final.sh $T || exit 1
export TMPDIR=/tmp
bash tools/gpu_prof.sh $T c2 2> gpurun_out/$T/prof2.log || { tail -30 gpurun_out/$T/prof2.log; exit 1; }
A=ntt-based-polynomial-multiplier-fpga_amd/apps/time_testing_gpu
for i in 1 2 3; do
  timeout -k 10 120 $A tests/golden/coeficientes_a.txt tests/golden/coeficientes_b.txt 2000 > gpurun_out/$T/time_testing_$i.txt 2>&1 || exit 1
  grep "us por" gpurun_out/$T/time_testing_$i.txt
done
timeout -k 10 120 python -c "import json, sys; sys.path.insert(0, '.'); from oracle import oracle as O; print(json.dumps({k: v * 1e6 for k, v in O.ref_anchors().items()}, indent=1))" > gpurun_out/$T/ref_anchors_us.json || exit 1
grep product4 gpurun_out/$T/ref_anchors_us.json
