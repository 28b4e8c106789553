set -e
B=tools/kbench/bin/kbench_base
mkdir -p gpurun_out
O=gpurun_out/stale_rows.txt
: > $O
timeout -k 5 60 $B 4096 2013265921 65536 300 >> $O
timeout -k 5 60 $B 4096 1073479681 65536 300 >> $O
timeout -k 5 60 $B 1024 2013265921 262144 300 >> $O
timeout -k 5 60 $B 1024 2013265921 4096 300 >> $O
timeout -k 5 60 $B 1024 1073479681 262144 300 >> $O
cat $O
