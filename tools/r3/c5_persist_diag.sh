# k_mp_persist diagnostics: per-task-type busy / wait times (NTTMUL_MP_STATS build), lag sweep,
# plain-policy variant (wrong hand-off, timing only)
set -o pipefail
OUT=gpurun_out/${1:-r3_c5d}; mkdir -p $OUT
B=tools/kbench/bin
{
for lag in 0 64 128 256; do echo -n "c5 lag=$lag "; KB_MP_LAG=$lag timeout -k 5 60 $B/kbench_c5 65536 4611686018425815041 1024 40 || exit 1; done
for lag in 16 64 256; do echo -n "stats lag=$lag "; KB_MP_LAG=$lag timeout -k 5 60 $B/kbench_c5stats 65536 4611686018425815041 1024 20 || exit 1; done
for lag in 64 256; do echo -n "plain lag=$lag "; KB_MP_LAG=$lag timeout -k 5 60 $B/kbench_c5plain 65536 4611686018425815041 1024 40 || exit 1; done
} > $OUT/diag.txt 2>&1
cat $OUT/diag.txt
