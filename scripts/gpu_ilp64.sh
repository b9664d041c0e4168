#!/bin/bash
# CRC64NVME two-chain streaming scan: GPU suite on the new build, then A/B (ab/libA.so = before,
# ab/libB.so = after) on C5, the C4 shard (131072 x 8 KiB) and 65536 x 16 KiB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${TAG:-ilp64}; mkdir -p $O; export TMPDIR=/tmp
cp ab/libB.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so &&
bash scripts/gpu_step.sh 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS:-} &&
tail -2 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
X="--steps 12 --warmup 2 --batches 2 --coalesce 1 --timing-launches 8 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0" &&
TAG=${TAG:-ilp64}/c5 REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 $X &&
TAG=${TAG:-ilp64}/c4 REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 131072 --buffer-bytes 8192 $X &&
TAG=${TAG:-ilp64}/k16 REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 65536 --buffer-bytes 16384 $X &&
echo "session ok"
