#!/bin/bash
# Round-3 session v16: crc64_xcd_kernel in 1024-thread workgroups (K, one per CU) vs 512 (A, two per
# CU): CRC64 parity on K, isolated C5 launches, then the config legs (3-stream pipelines).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v16}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
Q="--no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
cp ab/libK.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
bash scripts/gpu_step.sh 300 $O/pytest_K.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "crc64 or C5 or c5" --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest_K.log && grep -q " passed" $O/pytest_K.log && ! grep -q "failed" $O/pytest_K.log || { cp ab/libA.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so; exit 1; }
TAG=$T/c5 VARIANTS="A K" REPS=3 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 24 --warmup 4 --timing-launches 8 --only-coalesced $Q &&
VARIANTS="A K" TAG=$T/legs bash scripts/gpu_r03_v9.sh
