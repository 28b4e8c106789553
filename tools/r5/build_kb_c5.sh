#!/bin/bash
# kbench binaries for the round-5 C5 session (tools/r5/gpu_r5a.sh): the two splits of n = 65536
# (o_*: 16 x 4096, NTTMUL_C5_SQ=0; n_*: 256 x 256, NTTMUL_C5_SQ=1) and, for each, the
# intermediates' stores / loads redirected into one polynomial's worth of data (L2-resident):
#   st: the row pass's stores (tc) and the forward column pass's stores (ta, tb)
#   ld: the row pass's loads (ta, tb) and the inverse column pass's loads (tc)
#   ldst: both; all: both plus the forward column pass's loads (a, b)
# stpl / basepl: the same with plain (not non-temporal) column-pass loads and stores.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
export KB_FLAGS="-DKB_SET=2"
O="-DNTTMUL_C5_SQ=0"; N="-DNTTMUL_C5_SQ=1"
OST="-DKB_ABL_STROWS=16 -DKB_ABL_STCF=1"; OLD="-DKB_ABL_L2LOAD=16 -DKB_ABL_L2CI=1"
NST="-DKB_ABL_STROWS=256 -DKB_ABL_STCF=1"; NLD="-DKB_ABL_L2LOAD=256 -DKB_ABL_L2CI=1"
$R/tools/kbench/build.sh "o_base=$O" "o_st=$O $OST" "o_ld=$O $OLD" "o_ldst=$O $OST $OLD" \
  "o_all=$O $OST $OLD -DKB_ABL_L2CF=1" \
  "n_base=$N" "n_st=$N $NST" "n_ld=$N $NLD" "n_ldst=$N $NST $NLD" "n_all=$N $NST $NLD -DKB_ABL_L2CF=1" \
  "n_basepl=$N -DNTTMUL_NT_COLS=0" "n_stpl=$N $NST -DNTTMUL_NT_COLS=0"
