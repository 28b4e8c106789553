# NTTMUL_PRIO 1 (priority lowered at every forward exchange) / 2 (after the forward transform and
# after the base multiplication) vs oldest-first, at C2 and at other single-generation batches
set -o pipefail
OUT=gpurun_out/${1:-r3_prio2}; mkdir -p $OUT
B=tools/kbench/bin
run() { for v in base prio prio2; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v "$@" || exit 1; done; }
{
for i in 1 2; do KB_ROTATE=16 run 1024 2013265921 4096 2000; done
KB_ROTATE=16 run 1024 2013265921 8192 1000
KB_ROTATE=16 run 4096 2013265921 1024 1000
KB_ROTATE=16 run 4096 2013265921 2048 1000
KB_ROTATE=16 run 2048 2013265921 2048 1000
KB_ROTATE=16 run 512 2013265921 8192 2000
KB_ROTATE=16 run 256 2013265921 16384 2000
run 1024 2013265921 262144 50
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
