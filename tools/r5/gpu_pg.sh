#!/bin/bash
# Round-5 session D: C2 load order by generation (kbench KB_PRIO_GEN: the first generation of a
# one-generation launch issues its loads at the highest priority, later ones lower), against the
# library's issue-priority variant (KB_PRIO=0, automatic) and oldest-first issue (KB_PRIO=-1),
# three interleaved rounds over 16 rotated HBM buffer sets, 20,000 launches each.
set -o pipefail
OUT=gpurun_out/r5d; mkdir -p $OUT
export TMPDIR=/tmp
B=tools/kbench/bin
run() { echo -n "$1 "; shift; env "$@"; }
for i in 1 2 3; do
  for v in base noprio pg1024 pg2048 pg512; do
    case $v in
      noprio) echo -n "noprio "; KB_PRIO=-1 KB_ROTATE=16 timeout -k 5 60 $B/kbench_base 1024 2013265921 4096 20000 || exit 1 ;;
      *) echo -n "$v "; KB_ROTATE=16 timeout -k 5 60 $B/kbench_$v 1024 2013265921 4096 20000 || exit 1 ;;
    esac
  done
done 2>&1 | tee $OUT/pg.txt
echo done
