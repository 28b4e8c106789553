set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o c5 --output-format csv -- tools/kbench/bin/kbench_full 65536 4611686018425815041 1024 20 > gpurun_out/c5prof.log 2>&1
cat gpurun_out/c5prof.log | tail -2
find gpurun_out/c5prof -name "*stats*"
