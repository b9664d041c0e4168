#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/exp5; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
run e2 --branches 2 && run e3 --branches 3 && run e4 --branches 4 &&
AMDCRC_GRID_FRAC=0.5 run h2 --branches 2 && AMDCRC_GRID_FRAC=0.5 run h3 --branches 3 && AMDCRC_GRID_FRAC=0.5 run h4 --branches 4 &&
AMDCRC_GRID_FRAC=0.75 run q3 --branches 3 && AMDCRC_GRID_FRAC=0.75 run q4 --branches 4
