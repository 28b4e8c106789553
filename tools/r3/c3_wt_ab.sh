# C3: wave-typed layouts (NTTMUL_WAVE_TYPED=1: boundary differences left signed, permuted group
# layouts, wave-uniform branch) vs the round-2 layouts, interleaved; identical checksums required
set -o pipefail
OUT=gpurun_out/${1:-r3_wt}; mkdir -p $OUT
B=tools/kbench/bin
{
for i in 1 2 3 4; do for v in wt0 wt1; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v 4096 2013265921 65536 100 || exit 1; done; done
for v in wt0 wt1; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v 4096 1073479681 65536 100 || exit 1; done
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
