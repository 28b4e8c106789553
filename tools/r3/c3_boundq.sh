# C3: price of the boundary "+ q" (NTTMUL_ABL_BOUNDQ, wrong results), interleaved kbench A/B
set -o pipefail
OUT=gpurun_out/${1:-r3_bq}; mkdir -p $OUT
B=tools/kbench/bin
{
for i in 1 2 3 4; do for v in base boundq; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v 4096 2013265921 65536 100 || exit 1; done; done
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
