# stage loops by template recursion for 64-bit words (new) vs #pragma unroll everywhere (old):
# C5 rows lost a rolled loop; the 32-bit kernels keep their loops (C3 listing identical; the
# one-wave n = 1024 kernel's registers moved).  Interleaved kbench A/B.
set -o pipefail
OUT=gpurun_out/${1:-r3_unroll2}; mkdir -p $OUT
B=tools/kbench/bin
{
for i in 1 2 3; do for v in c5old c5new; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v 65536 4611686018425815041 1024 40 || exit 1; done; done
for i in 1 2; do for v in c3old base; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v 4096 2013265921 65536 100 || exit 1; done; done
for i in 1 2; do for v in c3old base; do echo -n "$v "; KB_ROTATE=16 timeout -k 5 60 $B/kbench_$v 1024 2013265921 4096 2000 || exit 1; done; done
for i in 1 2; do for v in c3old base; do echo -n "$v "; timeout -k 5 60 $B/kbench_$v 1024 2013265921 262144 50 || exit 1; done; done
} > $OUT/ab.txt 2>&1
cat $OUT/ab.txt
