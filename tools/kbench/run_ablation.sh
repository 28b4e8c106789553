set -e
cd $GRAFT_REPO_ROOT
B=tools/kbench/bin
for v in base noload noxchg nostore compute; do timeout -k 5 60 $B/kbench_$v 4096 2013265921 65536 20; done > gpurun_out/kb1.txt
for v in base noload; do timeout -k 5 60 $B/kbench_$v 1024 2013265921 65536 20; done >> gpurun_out/kb1.txt
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS -T --kernel-include-regex k_rows -d gpurun_out/pmc_stall -o st --output-format csv -- $B/kbench_base 4096 2013265921 65536 3 > gpurun_out/pmc_stall.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -T --kernel-include-regex k_rows -d gpurun_out/pmc_stall2 -o st2 --output-format csv -- $B/kbench_base 4096 2013265921 65536 3 > gpurun_out/pmc_stall2.log 2>&1
cat gpurun_out/kb1.txt
