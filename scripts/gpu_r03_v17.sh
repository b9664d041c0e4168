#!/bin/bash
# Round-3 session v17: s_setprio 1 for waves 4-7 of each workgroup (Y) vs release (A): C2 20-batch
# launch and C5 (crc64_xcd_kernel), isolated launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v17}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
Q="--no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
TAG=$T/c2 VARIANTS="A Y" REPS=3 bash scripts/ab_lib.sh python -u bench.py --gpus 1 --steps 20 --warmup 5 $Q &&
TAG=$T/c5 VARIANTS="A Y" REPS=3 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 24 --warmup 4 --timing-launches 8 --only-coalesced $Q &&
echo "session ok"
