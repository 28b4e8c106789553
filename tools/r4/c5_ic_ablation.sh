# C5 (n = 65536, 62-bit q, 1024 products, three launches): what the intermediates' round trips
# cost when they come from the Infinity Cache (MALL) or an XCD's L2 instead of HBM, by
# wrong-result kbench ablations (same instructions; the loads redirected): ic_* read polynomial
# p mod 32 (64 MiB of inputs: Infinity-Cache-resident), l2all reads one polynomial's worth
# (L2-resident) in all three passes.  acc = the product as built (the reference point).
# Interleaved, 3 rounds; then per-kernel times (rocprofv3 --stats) of acc, ic_all and l2all.
set -o pipefail
OUT=gpurun_out/${1:-r4_c5ic}; mkdir -p $OUT
export TMPDIR=/tmp
B=tools/kbench/bin
Q=4611686018425815041
for i in 1 2 3; do
  for v in c5acc c5ic_cf c5ic_ci c5ic_rows c5ic_all c5l2all; do
    timeout -k 5 60 $B/kbench_$v 65536 $Q 1024 200 || exit 1
  done
done 2>&1 | tee $OUT/ab.txt
for v in c5acc c5ic_all c5l2all; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o $v --output-format csv -- \
    $B/kbench_$v 65536 $Q 1024 200 > $OUT/prof_$v.log 2>&1 || exit 1
done
