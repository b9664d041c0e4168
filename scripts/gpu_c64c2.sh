#!/bin/bash
# C2-shape CRC64NVME: parity suite, then tile size (AMDCRC_SEG) / grid spread (AMDCRC_DEBUG bit 22)
# of crc64_stream4_kernel, and the C5 shape and C2 CRC32C as controls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-c64c2}; mkdir -p $O
# run TAG "ENV=.. ENV=.." bench-args...
run() { local tag=$1 envs=$2; shift 2; env X=0 $envs timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 --target-buffers 0 --steps 200 --warmup 20 "$@" > $O/$tag.log 2>&1 || return $?;
  grep '^{' $O/$tag.log | tail -1 > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); r=d['roofline']; print('%-18s' % '$tag', d['value'], 'GiB/s', d['pct_hbm_peak'], '% peak; kernel', r['kernel_ms'], 'frac', r['frac'])"; }
C5="--alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 40 --warmup 4 --timing-launches 8"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && tail -1 $O/pytest.log &&
run c2_crc64 "" --alg crc64nvme &&
run c2_crc64_spread "AMDCRC_DEBUG=4194304" --alg crc64nvme &&
run c2_crc64_seg512 "AMDCRC_SEG=512" --alg crc64nvme &&
run c2_crc32c "" &&
run c5_crc64 "" $C5
