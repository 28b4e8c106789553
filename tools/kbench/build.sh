#!/bin/bash
# Build kbench variants: tools/kbench/build.sh [VARIANT=-Dflags ...]
# (KB_OUT: output directory, default tools/kbench/bin; KB_FLAGS defaults to -DNTTMUL_KBENCH_LITE=1: only the n <= 4096, q < 2^31 product kernels;
#  KB_FLAGS=" " builds every kernel)
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
P=$R/ntt-based-polynomial-multiplier-fpga_amd
OUT=${KB_OUT:-$R/tools/kbench/bin}
mkdir -p $OUT
build() {
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$R/include -I$P/csrc -DNTTMUL_KBENCH_BUILD=1 -DVARIANT="\"$name\"" ${KB_FLAGS:--DNTTMUL_KBENCH_LITE=1} "$@" \
    $R/tools/kbench/kbench.cpp $P/csrc/kernels.hip $P/csrc/planner.cpp -o $OUT/kbench_$name &
}
if [ $# -eq 0 ]; then set -- base; fi
for v in "$@"; do
  case $v in
    base) build base ;;
    noload) build noload -DNTTMUL_ABL_NOLOAD=1 ;;
    noxchg) build noxchg -DNTTMUL_ABL_NOXCHG=1 ;;
    nostore) build nostore -DNTTMUL_ABL_NOSTORE=1 ;;
    compute) build compute -DNTTMUL_ABL_NOLOAD=1 -DNTTMUL_ABL_NOXCHG=1 -DNTTMUL_ABL_NOSTORE=1 ;;
    *=*) name=${v%%=*}; flags=${v#*=}; build $name $flags ;;
    *) build $v ;;
  esac
done
wait
ls $OUT
