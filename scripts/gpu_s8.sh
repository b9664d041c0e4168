#!/bin/bash
# 512-byte-row streaming scan (AMDCRC_DEBUG bit 15): parity first, then C2/C3/C4 against the
# 256-byte-row kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-s8}; mkdir -p $O
AMDCRC_DEBUG=32768 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "crc32c and (config2 or fuzz_strided or strided_shapes)" > $O/pytest8.log 2>&1
rc=$?; tail -2 $O/pytest8.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; local ev=$2; shift 2; env $ev timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 --no-read-ceiling "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('%-22s' % '$tag', d['value'], 'GiB/s', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
C3="--buffers 16 --buffer-bytes 268435456 --batches 1 --steps 10 --warmup 2 --timing-launches 4"
C4="--buffers 131072 --buffer-bytes 8192 --batches 1 --steps 40 --warmup 4 --timing-launches 8"
run c2_row256 X=1 --steps 400 &&
run c2_row512 AMDCRC_DEBUG=32768 --steps 400 &&
run c3_row256 X=1 $C3 &&
run c3_row512 AMDCRC_DEBUG=32768 $C3 &&
run c4_row256 X=1 $C4 &&
run c4_row512 AMDCRC_DEBUG=32768 $C4 &&
run c2_row256_b X=1 --steps 400 &&
run c2_row512_b AMDCRC_DEBUG=32768 --steps 400
