# C2 per-wave phase timestamps (NTTMUL_WAVE_TRACE kbench build), HBM-rotated and IC-resident
set -o pipefail
OUT=gpurun_out/${1:-r3_c2t2}; mkdir -p $OUT
B=tools/kbench/bin
{
echo "rotated x16:"; KB_ROTATE=16 timeout -k 5 60 $B/kbench_trace 1024 2013265921 4096 200 || exit 1
echo "one set (IC):"; timeout -k 5 60 $B/kbench_trace 1024 2013265921 4096 200 || exit 1
echo "batch 16384 rotated x4:"; KB_ROTATE=4 timeout -k 5 60 $B/kbench_trace 1024 2013265921 16384 100 || exit 1
} > $OUT/trace.txt 2>&1
cat $OUT/trace.txt
