# C2 with the issue-priority variant (auto): a-before-b loads and transforms (NTTMUL_SPLIT_AB) vs
# the interleaved form, interleaved kbench A/B
set -o pipefail
OUT=gpurun_out/${1:-r3_splitp}; mkdir -p $OUT
B=tools/kbench/bin
{
for i in 1 2 3; do for v in base split; do echo -n "$v "; KB_ROTATE=16 timeout -k 5 60 $B/kbench_$v 1024 2013265921 4096 2000 || exit 1; done; done
for v in base split; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v 1024 2013265921 262144 50 || exit 1; done
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
