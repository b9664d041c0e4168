#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/crc64; mkdir -p $O
timeout -k 10 300 python -m pytest -q -x tests/test_gpu_parity.py tests/test_multipart.py -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; tail -3 $O/parity.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; timeout -k 10 180 python bench.py --no-cpu-baseline --e2e-batches 0 "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], 'GiB/s', d['ms_per_step'], 'ms/step', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
run c5_crc64 --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 20 --warmup 2 --timing-launches 4 &&
run c2_crc64 --alg crc64nvme &&
AMDCRC_DEBUG=2048 run c5_crc64_old --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 20 --warmup 2 --timing-launches 4
