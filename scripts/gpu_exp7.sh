#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/exp7; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
C3="--buffers 16 --buffer-bytes 268435456 --batches 1 --steps 12 --warmup 3 --timing-launches 4"
run b1 $C3 --branches 1 && run b2 $C3 --branches 2 && run b3 $C3 --branches 3 &&
AMDCRC_DEBUG=4096 run b3np $C3 --branches 3 && AMDCRC_DEBUG=4096 run b2np $C3 --branches 2 &&
run c4b1 --buffers 131072 --buffer-bytes 8192 --batches 1 --steps 40 --warmup 4 --timing-launches 8 --branches 1
