#!/bin/bash
# Every BASELINE.json config on one GPU (device-resident GiB/s + isolated-launch roofline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-cfg}; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 180 python bench.py --no-cpu-baseline --e2e-batches 0 "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], 'GiB/s', d['ms_per_step'], 'ms/step', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
run c2_crc32c &&
run c2_crc32 --alg crc32 &&
run c3_crc32c --buffers 16 --buffer-bytes 268435456 --batches 1 --steps 10 --warmup 2 --timing-launches 4 &&
run c3_crc32 --alg crc32 --buffers 16 --buffer-bytes 268435456 --batches 1 --steps 10 --warmup 2 --timing-launches 4 &&
run c4_shard --buffers 131072 --buffer-bytes 8192 --batches 1 --steps 40 --warmup 4 --timing-launches 8 &&
run c5_crc64 --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 20 --warmup 2 --timing-launches 4 &&
run c5_xxh64 --alg xxh64 --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 6 --warmup 2 --timing-launches 2 --branches 2 &&
run c2_crc64 --alg crc64nvme &&
run c2_xxh64 --alg xxh64 --steps 40 --warmup 4 --timing-launches 8 &&
run c2_xxh3 --alg xxh3_64 --steps 20 --warmup 4 --timing-launches 4
