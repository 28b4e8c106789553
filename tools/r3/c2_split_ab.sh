# C2: k_rows (a and b transformed together) vs NTTMUL_SPLIT_AB (a's loads and transform first)
set -o pipefail
OUT=gpurun_out/${1:-r3_c2s}; mkdir -p $OUT
B=tools/kbench/bin
{
for i in 1 2 3; do for v in base splitab; do echo -n "$v "; KB_ROTATE=16 timeout -k 5 60 $B/kbench_$v 1024 2013265921 4096 2000 || exit 1; done; done
for v in base splitab; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v 1024 2013265921 262144 50 || exit 1; done
for v in base splitab; do echo -n "$v "; KB_STREAMS=2 KB_ROTATE=16 timeout -k 5 60 $B/kbench_$v 1024 2013265921 4096 2000 || exit 1; done
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
