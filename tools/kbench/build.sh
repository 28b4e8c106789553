#!/bin/bash
# Build kbench variants: tools/kbench/build.sh [VARIANT=-Dflags ...]
# (KB_OUT: output directory, default tools/kbench/bin; KB_FLAGS defaults to -DKB_SET=1: the n <= 4096,
#  q < 2^31 product kernels; -DKB_SET=2: C5, 64-bit words at n = 65536.  Variants: -DKB_ABL_* pricing
#  switches (kb_kernels.hip), or any exact A/B macro of csrc/)
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
P=$R/ntt-based-polynomial-multiplier-fpga_amd
OUT=${KB_OUT:-$R/tools/kbench/bin}
mkdir -p $OUT
# (KB_PL=1 variants include the generated reordered-argument k_rows)
python3 $R/tools/kbench/gen_rows_pl.py
build() {
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$R/include -I$P/csrc -I$R/tools/kbench -I$R/tools/kbench/bin -DVARIANT="\"$name\"" ${KB_FLAGS:--DKB_SET=1} "$@" \
    $R/tools/kbench/kbench.cpp $R/tools/kbench/kb_kernels.hip $P/csrc/planner.cpp -o $OUT/kbench_$name &
}
if [ $# -eq 0 ]; then set -- base; fi
for v in "$@"; do
  case $v in
    base) build base ;;
    noload) build noload -DKB_ABL_NOLOAD=1 ;;
    noxchg) build noxchg -DKB_ABL_NOXCHG=1 ;;
    nostore) build nostore -DKB_ABL_NOSTORE=1 ;;
    compute) build compute -DKB_ABL_NOLOAD=1 -DKB_ABL_NOXCHG=1 -DKB_ABL_NOSTORE=1 ;;
    *=*) name=${v%%=*}; flags=${v#*=}; build $name $flags ;;
    *) build $v ;;
  esac
done
wait
ls $OUT
