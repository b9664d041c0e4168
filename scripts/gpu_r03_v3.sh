#!/bin/bash
# Round-3 session v3: timing-only XCD-window chunk order (V: results wrong, timing only) against the
# release build (A) at C5 (CRC64NVME 8 x 64 MiB), the north-star target (16 x 64 MiB CRC32C), C3 and C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v3}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
Q="--no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
V=${VARIANTS:-A V}
TAG=$T/c5 VARIANTS="$V" REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 24 --warmup 4 --timing-launches 8 --only-coalesced $Q &&
TAG=$T/t16 VARIANTS="$V" REPS=2 bash scripts/ab_lib.sh python -u bench.py --buffers 16 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 20 --warmup 2 --timing-launches 8 --only-coalesced $Q &&
TAG=$T/c3 VARIANTS="$V" REPS=2 bash scripts/ab_lib.sh python -u bench.py --buffers 16 --buffer-bytes 268435456 --batches 2 --coalesce 1 --steps 8 --warmup 2 --timing-launches 4 --only-coalesced $Q &&
TAG=$T/c2 VARIANTS="$V" REPS=2 bash scripts/ab_lib.sh python -u bench.py --gpus 1 --steps 20 --warmup 5 --only-coalesced $Q &&
echo "session ok"
