#!/bin/bash
# Round-3 validation session v1 (fresh container; the tree at 363016a):
#   1. the full GPU parity suite, smoke
#   2. the driver's exact bench command, and a rocprof kernel trace of it
#   3. A/B of the whole-rotation ring loops (A, in-tree) vs the round-2 loops (B) at C2 / C5 / C4 shard
#   4. the ragged-list probe: A vs C (round-2 list kernel)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v1}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
Q="--no-configs --no-cpu-baseline --e2e-batches 0"
step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
step 180 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && tail -1 $O/smoke.log &&
step 400 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 && grep '^{' $O/bench_driver.log | cut -c1-400 &&
(cd /tmp && step 420 $O/prof_driver.log rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5) &&
TAG=$T/c2 VARIANTS="A B" REPS=2 bash scripts/ab_lib.sh python -u bench.py --gpus 1 --steps 20 --warmup 5 $Q &&
TAG=$T/c5 VARIANTS="A B" REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 24 --warmup 4 --timing-launches 8 --only-coalesced $Q &&
TAG=$T/c4 VARIANTS="A B" REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 131072 --buffer-bytes 8192 --batches 2 --coalesce 1 --steps 12 --warmup 2 --timing-launches 6 --only-coalesced $Q &&
TAG=$T/lists VARIANTS="A C" REPS=2 LIBDIR=ab bash scripts/ab_listprobe.sh &&
echo "session ok"
