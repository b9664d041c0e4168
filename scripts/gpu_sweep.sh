#!/bin/bash
# C2 launch-shape sweep for the streaming scan (diagnostic env knobs, engine.cpp).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-sw}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 --steps 400 ${BARGS} > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('%-22s' % '$tag', d['value'], 'GiB/s', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
run seg256 X=1 &&
run seg512 AMDCRC_SEG=512 &&
run seg128 AMDCRC_SEG=128 &&
run seg1024 AMDCRC_SEG=1024 &&
run wpc2_256 AMDCRC_WG_PER_CU=2 &&
run seg256_again X=1 &&
run seg512_again AMDCRC_SEG=512 &&
run c3_seg_default X=1 --buffers 16 --buffer-bytes 268435456 --batches 1 --steps 10 --warmup 2 --timing-launches 4 &&
run c3_wpc1 AMDCRC_WG_PER_CU=1 --buffers 16 --buffer-bytes 268435456 --batches 1 --steps 10 --warmup 2 --timing-launches 4 &&
run c4_default X=1 --buffers 131072 --buffer-bytes 8192 --batches 1 --steps 40 --warmup 4 --timing-launches 8 &&
run c4_wpc1 AMDCRC_WG_PER_CU=1 --buffers 131072 --buffer-bytes 8192 --batches 1 --steps 40 --warmup 4 --timing-launches 8
