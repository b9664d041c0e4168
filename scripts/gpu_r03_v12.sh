#!/bin/bash
# Round-3 session v12: crc64_xcd_kernel chunk size: A = 4 groups (16 KiB, in tree), T = 2, O = 1
# (the X order of the read-order table, a jump per group); CRC64 parity on O, then C5 kernel timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v12}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
Q="--no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
cp ab/libO.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
bash scripts/gpu_step.sh 300 $O/pytest_O.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "crc64 or C5 or c5" --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest_O.log && grep -q " passed" $O/pytest_O.log && ! grep -q "failed" $O/pytest_O.log || { cp ab/libA.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so; exit 1; }
TAG=$T/c5 VARIANTS="A T O" REPS=3 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 24 --warmup 4 --timing-launches 8 --only-coalesced $Q &&
echo "session ok"
