# C5 (n = 65536, 62-bit q, 1024 products): the three passes as a sub-batch pipeline over two
# streams (row passes on one, column passes on the other, ring of three scratch sets; kbench
# KB_SUB), with and without capping the row pass at 3 workgroups per CU (KB_ROWS_LDS: 6,400 B of
# extra LDS per row workgroup, 41,216 B in all, so 4 no longer fit the CU's 160 KiB and a
# column-pass workgroup (no LDS, <= 152 free VGPRs per SIMD) can be resident beside three row
# workgroups).  Interleaved, 3 rounds, one box; identical checksums expected.
set -o pipefail
OUT=gpurun_out/${1:-r4_c5pipe}; mkdir -p $OUT
B=tools/kbench/bin/kbench_c5pipe
Q=4611686018425815041
run() { echo "== $1"; shift; timeout -k 5 60 env "$@" $B 65536 $Q 1024 200 || exit 1; }
for i in 1 2 3; do
  run base KB_SUB=0
  echo "== base_noacc"; timeout -k 5 60 tools/kbench/bin/kbench_c5base 65536 $Q 1024 200 || exit 1
  run rows3 KB_ROWS_LDS=6400
  run sub128 KB_SUB=128
  run sub128_rows3 KB_SUB=128 KB_ROWS_LDS=6400
  run sub64_rows3 KB_SUB=64 KB_ROWS_LDS=6400
  run sub256_rows3 KB_SUB=256 KB_ROWS_LDS=6400
done 2>&1 | tee $OUT/ab.txt
