#!/bin/bash
# Every algorithm at the C2, C4-shard and C5 shapes (device-resident, one stream, roofline from the
# timed launches).  Outputs gpurun_out/${TAG:-matrix}/<alg>_<shape>.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-matrix}; mkdir -p $O
B="--no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling --branches 1 --only-coalesced --timing-launches 6"
for alg in crc32 crc32c crc64nvme xxh64 xxh3_64 xxh3_128; do
  for shape in "c2 1024 65536 20" "c4 131072 8192 20" "c5 8 67108864 6"; do
    set -- $shape
    st=$4; [ $alg = xxh64 ] && [ $1 = c5 ] && st=2
    bash scripts/gpu_step.sh 200 $O/${alg}_$1.log python -u bench.py --alg $alg --buffers $2 --buffer-bytes $3 --steps $st --warmup 2 $B || exit 1
    grep '^{' $O/${alg}_$1.log > $O/${alg}_$1.json
    python3 -c "import json; d=json.load(open('$O/${alg}_$1.json')); print('$alg $1', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
  done
done
echo "matrix ok"
