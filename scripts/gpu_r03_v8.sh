#!/bin/bash
# Round-3 session v8: crc64_rows16_kernel sets in XCD-window order (A, in tree) vs contiguous (Z):
# the rows16 parity tests, then the C4 shard CRC64NVME timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v8}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
Q="--no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
step 300 $O/pytest_r16.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "rows16 or shard or crc64" --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -2 $O/pytest_r16.log && grep -q " passed" $O/pytest_r16.log && ! grep -q "failed" $O/pytest_r16.log &&
TAG=$T/c4 VARIANTS="A Z" REPS=3 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 131072 --buffer-bytes 8192 --batches 2 --coalesce 1 --steps 12 --warmup 2 --timing-launches 6 --only-coalesced $Q &&
echo "session ok"
