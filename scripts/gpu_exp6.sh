#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/exp6; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
AMDCRC_GRID_FRAC=0.5 run h3 --branches 3 && AMDCRC_GRID_FRAC=0.5 run h3b16 --branches 3 --batches 16 &&
AMDCRC_GRID_FRAC=0.5 run h6 --branches 6 --batches 12 &&
AMDCRC_GRID_FRAC=0.333 run t4 --branches 4 && AMDCRC_GRID_FRAC=0.333 run t5 --branches 5 --batches 10 &&
AMDCRC_GRID_FRAC=0.25 run f5 --branches 5 --batches 10 && AMDCRC_GRID_FRAC=0.25 run f6 --branches 6 --batches 12 &&
AMDCRC_GRID_FRAC=0.5 run h3c3 --branches 3 --buffers 16 --buffer-bytes 268435456 --batches 3 --steps 12 --warmup 3 --timing-launches 4 &&
run f3c3 --branches 2 --buffers 16 --buffer-bytes 268435456 --batches 2 --steps 12 --warmup 2 --timing-launches 4
