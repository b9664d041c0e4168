#!/bin/bash
# Round-3 session v27: mid-size strided CRC64NVME batches (main regions below the XCD scan's 4 MiB):
# A = release (crc64_stream4_kernel), X = crc64_xcd_kernel from 2 chunks (-DAMDCRC_XCD_MIN_CHUNKS=2),
# B = crc64_braid_kernel (-DAMDCRC_XP_STREAM64=0); CRC64 parity on X and B first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v27}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
Q="--no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
cp ab/libA.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
bash scripts/gpu_step.sh 200 $O/pytest_lists_A.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "long_buffers_cut or ragged_list or front_pads" --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest_lists_A.log && grep -q " passed" $O/pytest_lists_A.log && ! grep -q "failed" $O/pytest_lists_A.log || exit 1
for v in X B; do
  cp ab/lib$v.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
  bash scripts/gpu_step.sh 300 $O/pytest_$v.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "crc64 or C5 or c5 or strided" --timeout 120 --timeout-method thread -p no:cacheprovider &&
  tail -1 $O/pytest_$v.log && grep -q " passed" $O/pytest_$v.log && ! grep -q "failed" $O/pytest_$v.log || exit 1
done
for shape in "4096 65536" "1024 65536" "256 1048576" "64 2097152"; do
  set -- $shape
  TAG=$T/s$1x$2 VARIANTS="A X B" REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers $1 --buffer-bytes $2 --batches 2 --coalesce 1 --steps 24 --warmup 4 --timing-launches 8 --only-coalesced $Q || exit 1
done
echo "session ok"
