#!/bin/bash
# BASELINE.json north_star target shape: CRC32C over batches of 64 MiB device-resident buffers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-tgt}; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 180 python bench.py --no-cpu-baseline --e2e-batches 0 "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); r=d['roofline']; print('%-16s' % '$tag', d['value'], 'GiB/s', d['pct_hbm_peak'], '% peak; kernel', r['kernel_ms'], 'frac', r['frac'], 'ceiling', r['read_ceiling'] and r['read_ceiling']['pipelined_gibs'])"; }
run t8x64_crc32c --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 30 --warmup 3 --timing-launches 6 &&
run t16x64_crc32c --buffers 16 --buffer-bytes 67108864 --batches 2 --steps 20 --warmup 3 --timing-launches 6 &&
run t64x64_crc32c --buffers 64 --buffer-bytes 67108864 --batches 1 --steps 6 --warmup 2 --timing-launches 3
