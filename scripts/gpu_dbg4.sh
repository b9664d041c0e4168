#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() { echo "== AMDCRC_DEBUG=${AMDCRC_DEBUG:-0} $*"; timeout -k 10 150 "$@" 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
G="--buffers 16 --buffer-bytes 67108864 --batches 2 --steps 60 --warmup 5 --no-cpu-baseline --timing-launches 16"
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider 2>&1 | tail -2 &&
run python bench.py $G &&
AMDCRC_DEBUG=8 run python bench.py $G &&
run python bench.py --steps 400 --no-cpu-baseline &&
AMDCRC_DEBUG=8 run python bench.py --steps 400 --no-cpu-baseline &&
run python bench.py --steps 400 --no-cpu-baseline --buffers 16 --buffer-bytes 4194304
