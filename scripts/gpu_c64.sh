#!/bin/bash
# GPU parity tests, then streaming vs braided scans on the C5 CRC64NVME shape, the C2 shape (both
# widths) and C3/C4 (CRC32C).  AMDCRC_DEBUG=16384 selects the pre-streaming kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-c64}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; local ev=$2; shift 2; env $ev timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('%-22s' % '$tag', d['value'], 'GiB/s', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
C5="--alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 20 --warmup 2 --timing-launches 4"
C3="--buffers 16 --buffer-bytes 268435456 --batches 1 --steps 10 --warmup 2 --timing-launches 4"
C4="--buffers 131072 --buffer-bytes 8192 --batches 1 --steps 40 --warmup 4 --timing-launches 8"
run c5_stream X=1 $C5 &&
run c5_braid AMDCRC_DEBUG=16384 $C5 &&
run c2_64_stream X=1 --alg crc64nvme --steps 300 &&
run c2_64_braid AMDCRC_DEBUG=16384 --alg crc64nvme --steps 300 &&
run c2_32c X=1 --steps 400 &&
run c3_32c X=1 $C3 &&
run c4_32c X=1 $C4 &&
run c2_32c_again X=1 --steps 400
