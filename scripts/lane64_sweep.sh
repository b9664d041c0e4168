#!/bin/bash
# CRC64NVME strided batches of short buffers: braided stream scan (ab/libA.so) vs lane-per-buffer
# (ab/libB.so) at 4..256 KiB per buffer, 512 MiB per step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-lane64}; mkdir -p $O
for L in ${SIZES:-4096 8192 16384 32768}; do
  n=$((${STEP:-1073741824} / L))
  for v in A B; do
    cp ab/lib$v.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
    bash scripts/gpu_step.sh 200 $O/${v}_$L.log python -u bench.py --alg ${ALG:-crc64nvme} --buffers $n --buffer-bytes $L --batches 2 --coalesce 1 --steps 8 --warmup 2 --timing-launches 6 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling || exit 1
    echo "$L $v $(grep '^{' $O/${v}_$L.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["roofline"]["frac"], d["roofline"]["kernel_ms"])')"
  done
done
cp ab/libA.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so
