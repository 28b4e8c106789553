# C2 under the issue-priority variant: generation stagger (NTTMUL_STAGGER x 512 cycles per
# generation of one-wave blocks before the loads) vs none, interleaved kbench A/B
set -o pipefail
OUT=gpurun_out/${1:-r3_stgp}; mkdir -p $OUT
B=tools/kbench/bin
{
for i in 1 2; do for v in base stg1 stg2 stg4; do echo -n "$v "; KB_ROTATE=16 timeout -k 5 60 $B/kbench_$v 1024 2013265921 4096 2000 || exit 1; done; done
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
