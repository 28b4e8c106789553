# C2: k_rows (one-wave blocks) vs k_rows_ab (two waves per product, KB_PIPE=-2), rotated
set -o pipefail
OUT=gpurun_out/${1:-r3_c2ab}; mkdir -p $OUT
B=tools/kbench/bin
{
for i in 1 2 3; do for p in 0 -2; do echo -n "pipe=$p "; KB_PIPE=$p KB_ROTATE=16 timeout -k 5 60 $B/kbench_base 1024 2013265921 4096 2000 || exit 1; done; done
for p in 0 -2; do echo -n "pipe=$p "; KB_PIPE=$p timeout -k 5 60 $B/kbench_base 1024 2013265921 262144 50 || exit 1; done
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
