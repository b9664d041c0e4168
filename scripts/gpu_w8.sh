#!/bin/bash
# W=32 streaming scan on 8-byte words: GPU suite on the new build, then A/B (ab/libA.so = 4-byte
# words, ab/libB.so = 8-byte words) on the driver-shaped C2 run, C3, the target shape and the C4 shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${TAG:-w8}; mkdir -p $O; export TMPDIR=/tmp
cp ab/libB.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so &&
bash scripts/gpu_step.sh 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS:-} &&
tail -2 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
TAG=${TAG:-w8}/c2 REPS=3 bash scripts/ab_lib.sh python -u bench.py --steps 20 --warmup 5 --no-configs --e2e-batches 0 --no-cpu-baseline &&
X="--steps 12 --warmup 2 --batches 2 --coalesce 1 --timing-launches 8 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0" &&
TAG=${TAG:-w8}/c3 REPS=2 bash scripts/ab_lib.sh python -u bench.py --buffers 16 --buffer-bytes 268435456 $X &&
TAG=${TAG:-w8}/t16 REPS=2 bash scripts/ab_lib.sh python -u bench.py --buffers 16 --buffer-bytes 67108864 $X &&
TAG=${TAG:-w8}/c4 REPS=2 bash scripts/ab_lib.sh python -u bench.py --buffers 131072 --buffer-bytes 8192 $X &&
echo "session ok"
