# C3 / C2: LDS exchanges vs the register/lane transposes of an intra-wave (one-wave-per-product)
# exchange (NTTMUL_ABL_PERMXCHG, wrong results) vs no exchange at all (NTTMUL_ABL_NOXCHG),
# interleaved kbench A/B, then SQ_INSTS_VALU / SQ_WAVES of each C3 variant
set -o pipefail
OUT=gpurun_out/${1:-r3_permx}; mkdir -p $OUT
B=tools/kbench/bin
{
for i in 1 2 3 4; do for v in base permx noxchg; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v 4096 2013265921 65536 100 || exit 1; done; done
for i in 1 2; do for v in base permx noxchg; do echo -n "$v "; KB_ROTATE=16 timeout -k 5 60 $B/kbench_$v 1024 2013265921 4096 2000 || exit 1; done; done
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
cd /tmp && export TMPDIR=/tmp
for v in base permx noxchg; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -d $GRAFT_REPO_ROOT/$OUT/pmc_$v -o pmc -- $GRAFT_REPO_ROOT/$B/kbench_$v 4096 2013265921 65536 5 > $GRAFT_REPO_ROOT/$OUT/pmc_$v.log 2>&1 || exit 1
done
