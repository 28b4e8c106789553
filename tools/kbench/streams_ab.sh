set -o pipefail
for i in 1 2 3; do for s in 1 2; do echo -n "streams=$s "; KB_STREAMS=$s timeout -k 5 60 tools/kbench/bin/kbench_base 1024 2013265921 4096 1000 || exit 1; done; done
for i in 1 2; do for s in 1 2; do echo -n "streams=$s "; KB_STREAMS=$s timeout -k 5 60 tools/kbench/bin/kbench_base 4096 2013265921 65536 100 || exit 1; done; done
