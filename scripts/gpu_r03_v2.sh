#!/bin/bash
# Round-3 session v2: W=32 streaming-scan issue experiments (A = in-tree release; I = the next slot's
# eight loads issued at row 0; R = a four-slot ring; J = both) at the C2 driver shape, the north-star
# target shape and C3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v2}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
Q="--no-configs --no-cpu-baseline --e2e-batches 0"
V=${VARIANTS:-A I R J}
TAG=$T/c2 VARIANTS="$V" REPS=2 bash scripts/ab_lib.sh python -u bench.py --gpus 1 --steps 20 --warmup 5 $Q &&
TAG=$T/t16 VARIANTS="$V" REPS=2 bash scripts/ab_lib.sh python -u bench.py --buffers 16 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 20 --warmup 2 --timing-launches 8 --only-coalesced $Q &&
TAG=$T/c3 VARIANTS="$V" REPS=2 bash scripts/ab_lib.sh python -u bench.py --buffers 16 --buffer-bytes 268435456 --batches 2 --coalesce 1 --steps 8 --warmup 2 --timing-launches 4 --only-coalesced $Q &&
echo "session ok"
