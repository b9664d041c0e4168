#!/bin/bash
# Round-3 session v4: CRC64NVME C5 / C4 shard, A (release) vs I (issue-ahead loads) vs V (timing-only
# XCD-window chunk order) vs W (both)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v4}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
Q="--no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
V=${VARIANTS:-A I V W}
TAG=$T/c5 VARIANTS="$V" REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 24 --warmup 4 --timing-launches 8 --only-coalesced $Q &&
TAG=$T/c4 VARIANTS="A I" REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 131072 --buffer-bytes 8192 --batches 2 --coalesce 1 --steps 12 --warmup 2 --timing-launches 6 --only-coalesced $Q &&
echo "session ok"
