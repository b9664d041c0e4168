#!/bin/bash
# CRC64NVME 4-copy / two-workgroups-per-CU streaming scan (AMDCRC_DEBUG bit 20): parity, then C5
# and the C2 shape against the 8-copy kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-c64b}; mkdir -p $O
AMDCRC_DEBUG=1048576 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "crc64nvme and (config2 or fuzz_strided or strided_shapes or config5)" > $O/pytest4.log 2>&1
rc=$?; tail -1 $O/pytest4.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; local ev=$2; shift 2; env $ev timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 --no-read-ceiling "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('%-22s' % '$tag', d['value'], 'GiB/s', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
C5="--alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 20 --warmup 2 --timing-launches 4"
run c5_copies8 X=1 $C5 &&
run c5_copies4 AMDCRC_DEBUG=1048576 $C5 &&
run c2_64_copies8 X=1 --alg crc64nvme --steps 300 &&
run c2_64_copies4 AMDCRC_DEBUG=1048576 --alg crc64nvme --steps 300 &&
run c5_copies8_b X=1 $C5 &&
run c5_copies4_b AMDCRC_DEBUG=1048576 $C5
