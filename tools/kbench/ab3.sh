#!/bin/bash
# 3 interleaved kbench runs of each variant in $VARIANTS (default: base mont): ab3.sh <kbench args>
B=$(dirname "$0")/bin
for i in 1 2 3; do for v in ${VARIANTS:-base mont}; do
  timeout -k 5 60 $B/kbench_$v "$@" || exit 1
done; done
