#!/bin/bash
# Round-3 session v5: crc64_xcd_kernel (A = in-tree, 4-group chunks; E = 8-group chunks; Z = the
# round-2 crc64_stream4_kernel path): the CRC64NVME parity tests, then C5 timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v5}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
Q="--no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
step 300 $O/pytest_xcd.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "crc64 or C5 or c5 or multi_batch" --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -2 $O/pytest_xcd.log && grep -q " passed" $O/pytest_xcd.log && ! grep -q "failed" $O/pytest_xcd.log &&
TAG=$T/c5 VARIANTS="A E Z" REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 24 --warmup 4 --timing-launches 8 --only-coalesced $Q &&
echo "session ok"
