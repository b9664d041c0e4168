#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/exp3; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
export AMDCRC_DEBUG=${DBG:-256}
run e1 --mode eager --branches 1 &&
run e2 --mode eager --branches 2 &&
run e3 --mode eager --branches 3 &&
run e4 --mode eager --branches 4 &&
run e4b16 --mode eager --branches 4 --batches 16 &&
run e8 --mode eager --branches 8 --batches 16
