#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pool; mkdir -p $O
timeout -k 10 300 python -m pytest -q -x tests/test_gpu_parity.py tests/test_multipart.py -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; tail -3 $O/parity.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; timeout -k 10 180 python bench.py --no-cpu-baseline --e2e-batches 0 "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], 'GiB/s', d['ms_per_step'], 'ms/step', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
for dbg in 0 4096; do
  export AMDCRC_DEBUG=$dbg
  run c2_$dbg &&
  run c3_$dbg --buffers 16 --buffer-bytes 268435456 --batches 1 --steps 10 --warmup 2 --timing-launches 4 &&
  run c4_$dbg --buffers 131072 --buffer-bytes 8192 --batches 1 --steps 40 --warmup 4 --timing-launches 8 &&
  timeout -k 10 120 python aws-crt-cpp_amd/tools/timeline.py > $O/tl_$dbg.log 2>&1 && sed -n 2,8p $O/tl_$dbg.log || exit 1
done
