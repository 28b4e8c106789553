# C2: issue priority lowered as a wave completes transform groups (NTTMUL_PRIO) vs oldest-first,
# interleaved kbench A/B, then the per-SIMD trace of the prio build
set -o pipefail
OUT=gpurun_out/${1:-r3_prio}; mkdir -p $OUT
B=tools/kbench/bin
{
for i in 1 2 3; do for v in base prio; do echo -n "$v "; KB_ROTATE=16 timeout -k 5 60 $B/kbench_$v 1024 2013265921 4096 2000 || exit 1; done; done
for v in base prio; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v 1024 2013265921 262144 50 || exit 1; done
for v in base prio; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v 4096 2013265921 65536 100 || exit 1; done
echo "prio trace rotated x16:"; KB_ROTATE=16 timeout -k 5 60 $B/kbench_prtrace 1024 2013265921 4096 200 || exit 1
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
