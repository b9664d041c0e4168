#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
run() { echo "== $*"; timeout -k 10 150 "$@" 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
G="--buffers 16 --buffer-bytes 67108864 --batches 2 --steps 60 --warmup 5 --no-cpu-baseline --timing-launches 16"
run python bench.py $G &&
AMDCRC_DEBUG=1 run python bench.py $G &&
run python bench.py --buffers 1 --buffer-bytes 1073741824 --batches 2 --steps 60 --warmup 5 --no-cpu-baseline --timing-launches 16 &&
run python bench.py --steps 400 --no-cpu-baseline &&
AMDCRC_DEBUG=1 run python bench.py --steps 400 --no-cpu-baseline &&
timeout -k 10 100 aws-crt-cpp_amd/build/tools/overlapbench 1 1024 1 | grep -E "R |M |dword" &&
timeout -k 10 100 aws-crt-cpp_amd/build/tools/overlapbench 1 64 2 | grep -E "dword|R real" &&
G="--buffers 16 --buffer-bytes 67108864 --batches 2 --steps 60 --warmup 5 --no-cpu-baseline --timing-launches 16"
AMDCRC_DEBUG=4 run python bench.py $G && AMDCRC_DEBUG=4 run python bench.py --steps 400 --no-cpu-baseline
