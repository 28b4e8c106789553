# C2 (n=1024 x 4096, one generation of one-wave blocks): base vs load stagger by generation,
# buffers rotated over 16 sets (HBM), interleaved; plus C5 DRAM-vs-fabric read requests for the
# three-launch and persistent forms (MALL hits = RDREQ - RDREQ_DRAM).
set -o pipefail
OUT=gpurun_out/${1:-r3_c2st}; mkdir -p $OUT
export TMPDIR=/tmp
B=tools/kbench/bin
{
for i in 1 2 3; do for v in base st2 st4 st8; do echo -n "$v "; KB_ROTATE=16 timeout -k 5 60 $B/kbench_$v 1024 2013265921 4096 2000 || exit 1; done; done
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
for lag in 0 256; do
  KB_MP_LAG=$lag timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum -d $OUT/pmc_lag$lag -o pmc --output-format csv -- $B/kbench_c5 65536 4611686018425815041 1024 5 > $OUT/pmc_lag$lag.log 2>&1 || { tail -5 $OUT/pmc_lag$lag.log; exit 1; }
done
find $OUT -name "*counter_collection*" | head
