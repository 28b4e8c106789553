#!/bin/bash
# Device-resident rate of the product kernels over (n, q, batch) with the full kbench build
# (tools/kbench/build.sh full, KB_FLAGS=" "): DESIGN.md §5 "Other configurations"
set -o pipefail
B=tools/kbench/bin/kbench_full
O=gpurun_out/config_table.txt
mkdir -p gpurun_out
: > $O
run() { timeout -k 5 90 $B "$@" >> $O || { echo "FAILED $*" >> $O; exit 1; }; }
run 4096 2013265921 65536 300          # C3 (Arith32P3)
run 4096 1073479681 65536 300          # 30-bit q (Arith32H)
run 4096 4293918721 65536 200          # full 32-bit q (Arith32W)
run 2048 2013265921 131072 300
run 1024 2013265921 262144 300
run 1024 1073479681 262144 300
run 512 2013265921 524288 300
run 256 2013265921 1048576 300
run 8192 2013265921 32768 200         # multi-pass, 32-bit words
run 65536 2013265921 1024 200         # multi-pass n = 65536, 31-bit q
run 65536 4293918721 1024 200         # n = 65536, full 32-bit q
run 65536 4611686018425815041 1024 100  # C5
run 4096 4611686018425815041 65536 100  # 62-bit q at n = 4096 (Arith64)
cat $O
