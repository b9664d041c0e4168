#!/bin/bash
# Prologue-order experiment (AMDCRC_DEBUG 32: tables first; 64: group 0, tables, group 1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/exp2; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
for dbg in ${DBGS:-0 32 64}; do
  export AMDCRC_DEBUG=$dbg
  run "g2_$dbg" --branches 2 &&
  run "e2_$dbg" --mode eager --branches 2 &&
  run "big_$dbg" --buffers 16 --buffer-bytes 67108864 --batches 2 --steps 40 --warmup 4 --timing-launches 8 &&
  timeout -k 10 120 python aws-crt-cpp_amd/tools/timeline.py > $O/tl_$dbg.log 2>&1 && sed -n 2,8p $O/tl_$dbg.log || exit 1
done
