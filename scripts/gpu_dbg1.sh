#!/bin/bash
# timing decomposition of the product scan kernel (AMDCRC_DEBUG skips pieces; results invalid)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
run() { echo "== $*"; timeout -k 10 150 "$@" 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
run python bench.py --steps 400 --no-cpu-baseline &&
AMDCRC_DEBUG=1 run python bench.py --steps 400 --no-cpu-baseline &&
AMDCRC_DEBUG=2 run python bench.py --steps 400 --no-cpu-baseline &&
run python bench.py --steps 400 --no-cpu-baseline --buffers 16 --buffer-bytes 4194304 &&
AMDCRC_DEBUG=1 run python bench.py --steps 400 --no-cpu-baseline --buffers 16 --buffer-bytes 4194304 &&
run python bench.py --steps 100 --no-cpu-baseline --buffers 16 --buffer-bytes 67108864 --batches 2
