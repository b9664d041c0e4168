#!/bin/bash
# C2 launch-shape sweep for the streaming scan (diagnostic env knobs, engine.cpp).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-sw}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 --steps 400 ${BARGS} > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('%-22s' % '$tag', d['value'], 'GiB/s', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
run pool256 X=1 &&
run static512 AMDCRC_DEBUG=4096 AMDCRC_SEG=512 &&
run pool128 AMDCRC_SEG=128 &&
run static256 AMDCRC_DEBUG=4096 &&
run pool64 AMDCRC_SEG=64 &&
run pool256_again X=1 &&
run static512_again AMDCRC_DEBUG=4096 AMDCRC_SEG=512 &&
timeout -k 10 60 python aws-crt-cpp_amd/tools/timeline.py > $O/timeline.log 2>&1 && head -12 $O/timeline.log
