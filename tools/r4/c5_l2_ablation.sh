# C5 (n = 65536, 62-bit q, 1024 products, three launches): what reading each pass's inputs from
# L2 instead of HBM saves, by wrong-result kbench ablations (the same instructions, the loads
# redirected to one polynomial's worth of data): rows (k_rows reads 16 rows = 1 MiB),
# CI (k_cols_inv reads polynomial 0), CF (k_cols_fwd reads polynomial 0), rows + CI.
# Interleaved, 3 rounds, one box.
set -o pipefail
OUT=gpurun_out/${1:-r4_c5l2}; mkdir -p $OUT
B=tools/kbench/bin
for i in 1 2 3; do
  for v in c5base c5l2rows c5l2ci c5l2cf c5l2rc; do
    timeout -k 5 60 $B/kbench_$v 65536 4611686018425815041 1024 200 || exit 1
  done
done 2>&1 | tee $OUT/ab.txt
