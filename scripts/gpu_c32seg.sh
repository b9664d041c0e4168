#!/bin/bash
# C2-shape CRC32C: stream tile size (AMDCRC_SEG 512 = 32 KiB default, 1024 = whole-buffer tiles).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-c32seg}; mkdir -p $O
run() { local tag=$1 envs=$2; shift 2; env X=0 $envs timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 --target-buffers 0 --steps 400 --warmup 20 "$@" > $O/$tag.log 2>&1 || return $?;
  grep '^{' $O/$tag.log | tail -1 > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); r=d['roofline']; print('%-18s' % '$tag', d['value'], 'GiB/s', d['pct_hbm_peak'], '% peak; kernel', r['kernel_ms'], 'frac', r['frac'])"; }
run base "" &&
run seg1024 "AMDCRC_SEG=1024" &&
run seg256 "AMDCRC_SEG=256" &&
run base2 "" &&
run seg1024b "AMDCRC_SEG=1024" &&
run crc32_base "" --alg crc32 &&
run crc32_seg1024 "AMDCRC_SEG=1024" --alg crc32
