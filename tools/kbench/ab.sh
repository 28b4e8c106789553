set -e
cd $GRAFT_REPO_ROOT
B=tools/kbench/bin
echo "== ${ARGS:-4096 2013265921 65536 50}" >> gpurun_out/ab.txt
for i in 1 2 3; do for v in $VARIANTS; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v ${ARGS:-4096 2013265921 65536 50}; done; done >> gpurun_out/ab.txt 2>&1
cat gpurun_out/ab.txt
