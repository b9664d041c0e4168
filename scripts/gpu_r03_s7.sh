#!/bin/bash
# Round-3 session 7: whole-rotation ring loops (no exit between the three steps of a rotation) in the
# streaming scans, and the list streaming scan (crc32_list_stream_kernel).  ab/libA.so = in-tree build.
#   1. the full GPU parity suite on A
#   2. C2 driver shape, C5 and C4-shard CRC64NVME: A vs B (B = the round-2 loops, AMDCRC_XP_RING_BREAKS)
#   3. ragged-list probe: A vs C (round-2 list kernel) vs D (list stream, 2 tiles per wave slot)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03s7}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
Q="--no-configs --no-cpu-baseline --e2e-batches 0"
step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
TAG=$T/c2 VARIANTS="A B" REPS=2 bash scripts/ab_lib.sh python -u bench.py --gpus 1 --steps 20 --warmup 5 $Q &&
TAG=$T/c5 VARIANTS="A B" REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 24 --warmup 4 --timing-launches 8 --only-coalesced $Q &&
TAG=$T/c4 VARIANTS="A B" REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 131072 --buffer-bytes 8192 --batches 2 --coalesce 1 --steps 12 --warmup 2 --timing-launches 6 --only-coalesced $Q &&
TAG=$T/lists VARIANTS="A C D" REPS=2 LIBDIR=ab bash scripts/ab_listprobe.sh &&
echo "session ok"
