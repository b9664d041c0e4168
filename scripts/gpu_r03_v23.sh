#!/bin/bash
# Round-3 session v23: crc64_xcd_kernel with front pads (buffer-resource loads, A) vs the previous
# whole-chunk version (P): CRC64 parity on A, C5 timing A / P, then a 64 MiB + 48 KiB + 16 B shape
# (A takes the XCD scan with a pad, P the stream4 / braided path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v23}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
Q="--no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
bash scripts/gpu_step.sh 300 $O/pytest_A.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "crc64 or C5 or c5 or graph" --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest_A.log && grep -q " passed" $O/pytest_A.log && ! grep -q "failed" $O/pytest_A.log || exit 1
TAG=$T/c5 VARIANTS="A P" REPS=3 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 24 --warmup 4 --timing-launches 8 --only-coalesced $Q &&
TAG=$T/pad VARIANTS="A P" REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67158032 --batches 2 --coalesce 1 --steps 24 --warmup 4 --timing-launches 8 --only-coalesced $Q &&
echo "session ok"
