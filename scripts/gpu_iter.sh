#!/bin/bash
# Quick iteration: GPU parity tests, then C2 / C3 / C4 / C5-CRC64 device-resident bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-it}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; timeout -k 10 180 python bench.py --no-cpu-baseline --e2e-batches 0 "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], 'GiB/s', d['ms_per_step'], 'ms/step', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])"; }
run c2_crc32c ${C2ARGS} &&
run c3_crc32c --buffers 16 --buffer-bytes 268435456 --batches 1 --steps 10 --warmup 2 --timing-launches 4 &&
run c4_shard --buffers 131072 --buffer-bytes 8192 --batches 1 --steps 40 --warmup 4 --timing-launches 8 &&
run c5_crc64 --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 20 --warmup 2 --timing-launches 4
