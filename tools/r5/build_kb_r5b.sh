#!/bin/bash
# kbench binaries for tools/r5/gpu_r5b.sh.  C5 (KB_SET=2): the square split with tiled
# intermediates (t_*, the library default), untiled (u_base) and the 16 x 4096 split (o_*), each
# with the intermediates' stores / loads redirected into one polynomial's worth of data
# (L2-resident; the store window is a polynomial apart from the load window):
#   st: row-pass stores (tc) + forward-column stores (ta, tb); ld: row-pass loads (ta, tb) +
#   inverse-column loads (tc); ldst: both; all: both + the forward column pass's loads (a, b).
# C3 (KB_SET=1): base and the no-load / no-store / no-exchange / compute-only pricing variants.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
rm -f $R/tools/kbench/bin/kbench_*
T="-DNTTMUL_C5_SQ=1 -DNTTMUL_C5_TILE=1"; U="-DNTTMUL_C5_SQ=1 -DNTTMUL_C5_TILE=0"; O="-DNTTMUL_C5_SQ=0"
NST="-DKB_ABL_STROWS=256 -DKB_ABL_STCF=1"; NLD="-DKB_ABL_L2LOAD=256 -DKB_ABL_L2CI=1"
OST="-DKB_ABL_STROWS=16 -DKB_ABL_STCF=1"; OLD="-DKB_ABL_L2LOAD=16 -DKB_ABL_L2CI=1"
KB_FLAGS="-DKB_SET=2" $R/tools/kbench/build.sh "t_base=$T" "u_base=$U" "o_base=$O" \
  "t_st=$T $NST" "t_ld=$T $NLD" "t_ldst=$T $NST $NLD" "t_all=$T $NST $NLD -DKB_ABL_L2CF=1" \
  "o_st=$O $OST" "o_ld=$O $OLD" "o_ldst=$O $OST $OLD" "o_all=$O $OST $OLD -DKB_ABL_L2CF=1" > /dev/null
KB_FLAGS="-DKB_SET=1" $R/tools/kbench/build.sh base noload nostore noxchg compute
