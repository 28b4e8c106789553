# Round-4 closing evidence on the final build: standalone-transform tests and lines, then the
# full GPU suite, smoke, C3 / C5 / C2 profiles (rocprof stats + PMC keyed to this code object),
# the driver's command, the C4 slice, the server and the reference anchors, and the --op lines.
set -o pipefail
T=${1:-r4final3}
bash tools/r4/gpu_xform.sh $T/xform || exit 1
bash tools/r4/gpu_final.sh $T || exit 1
bash tools/r4/gpu_final2.sh $T || exit 1
bash tools/r4/gpu_ops.sh $T/ops || exit 1
