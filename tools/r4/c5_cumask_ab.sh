# C5 (n = 65536, 62-bit q, 1024 products) as a sub-batch pipeline with the row and column passes
# on disjoint CU sets (kbench KB_SUB + KB_COL_CUS: CU-masked streams) instead of sharing every CU
# -- the co-residency problem of rounds 2-4 taken out of the picture.  Interleaved, 2 rounds, one
# box; identical checksums expected.
set -o pipefail
OUT=gpurun_out/${1:-r4_c5cumask}; mkdir -p $OUT
B=tools/kbench/bin/kbench_c5pipe
Q=4611686018425815041
run() { echo "== $1"; shift; timeout -k 5 60 env "$@" $B 65536 $Q 1024 200 || exit 1; }
for i in 1 2; do
  run base KB_SUB=0
  run sub256 KB_SUB=256
  for cus in 64 96 128; do
    run sub256_col$cus KB_SUB=256 KB_COL_CUS=$cus
    run sub128_col$cus KB_SUB=128 KB_COL_CUS=$cus
  done
done 2>&1 | tee $OUT/ab.txt
