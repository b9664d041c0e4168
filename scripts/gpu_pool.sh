#!/bin/bash
# Workgroup-pool streaming scan (AMDCRC_DEBUG bit 19): parity, then C2 against the static split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-pool}; mkdir -p $O
for sg in 128 256; do
AMDCRC_DEBUG=524288 AMDCRC_SEG=$sg timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "crc32c and (config2 or fuzz_strided or strided_shapes)" > $O/pytest_$sg.log 2>&1
rc=$?; tail -1 $O/pytest_$sg.log; [ $rc -eq 0 ] || exit $rc
done
run() { local tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 --no-read-ceiling --steps 400 > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('%-22s' % '$tag', d['value'], 'GiB/s', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
run static512 X=1 &&
run pool256 AMDCRC_DEBUG=524288 AMDCRC_SEG=256 &&
run pool128 AMDCRC_DEBUG=524288 AMDCRC_SEG=128 &&
run pool64 AMDCRC_DEBUG=524288 AMDCRC_SEG=64 &&
run static512_b X=1 &&
run pool128_b AMDCRC_DEBUG=524288 AMDCRC_SEG=128
