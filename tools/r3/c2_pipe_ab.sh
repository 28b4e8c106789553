# C2: k_rows (one product per one-wave block) vs k_rows_pipe (KB_PIPE products per wave, loads of
# the next product in flight during the current one's transforms, twiddles in LDS), 16 rotated
# buffer sets (HBM), interleaved, identical checksums; then n = 1024 x 262144 and C5 PMC.
set -o pipefail
OUT=gpurun_out/${1:-r3_c2p}; mkdir -p $OUT
export TMPDIR=/tmp
B=tools/kbench/bin
{
for i in 1 2 3; do for p in 0 1 2 4; do echo -n "pipe=$p "; KB_PIPE=$p KB_ROTATE=16 timeout -k 5 60 $B/kbench_base 1024 2013265921 4096 2000 || exit 1; done; done
for p in 0 2 4 8 16; do echo -n "pipe=$p "; KB_PIPE=$p timeout -k 5 60 $B/kbench_base 1024 2013265921 262144 50 || exit 1; done
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
for lag in 0 256; do
  KB_MP_LAG=$lag timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum -d $OUT/pmc_lag$lag -o pmc --output-format csv -- $B/kbench_c5 65536 4611686018425815041 1024 5 > $OUT/pmc_lag$lag.log 2>&1 || { tail -5 $OUT/pmc_lag$lag.log; exit 1; }
done
find $OUT -name "*counter_collection*"
