# C5 A/B: three launches (KB_MP_LAG=0) vs the persistent k_mp_persist at several lags, one box,
# interleaved; identical checksums required.
set -o pipefail
OUT=gpurun_out/${1:-r3_c5p}; mkdir -p $OUT
B=tools/kbench/bin/kbench_c5
for i in 1 2; do
  for lag in 0 8 16 32 64; do
    echo -n "lag=$lag "
    KB_MP_LAG=$lag timeout -k 5 60 $B 65536 4611686018425815041 1024 40 || exit 1
  done
done 2>&1 | tee $OUT/ab.txt
