set -o pipefail
tools/gpu_ab.sh r2i "base nopad2" "1024 2013265921 4096 1000" "base nopad2" "1024 2013265921 262144 100" "base nopad2" "512 2013265921 262144 100" || exit 1
tools/gpu_check.sh r2i || exit 1
STREAMS="1 2" tools/c2_streams.sh
