#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/exp4; mkdir -p $O
timeout -k 10 300 python -m pytest -q -x tests/test_gpu_parity.py tests/test_multipart.py -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; tail -2 $O/parity.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
for dbg in ${DBGS:-0 512}; do
  export AMDCRC_DEBUG=$dbg
  run "g2_$dbg" --branches 2 &&
  run "e1_$dbg" --mode eager --branches 1 &&
  run "e2_$dbg" --mode eager --branches 2 &&
  run "big_$dbg" --buffers 16 --buffer-bytes 67108864 --batches 2 --steps 40 --warmup 4 --timing-launches 8 &&
  timeout -k 10 120 python aws-crt-cpp_amd/tools/timeline.py > $O/tl_$dbg.log 2>&1 && sed -n 2,8p $O/tl_$dbg.log || exit 1
done
