#!/bin/bash
# Round-3 session 2: ab/libA.so (8-byte-word CRC32 scan, XXH64 host route), ab/libB.so (16-byte-word
# scan, chain lookups issued ahead of the off-chain XORs), ab/libC.so (A without the XXH64 host route).
#   1. GPU parity suite on A (streaming XXH3 on device chunks, the XXH64 host route, everything else)
#   2. A/B of the 16-byte-word scan: the driver-shaped C2 run (3 reps), the target shape (2 reps)
#   3. the XXH64 round's instruction costs on one wave (tools/chainbench)
#   4. hash paths on device data with A and C (tools/hash_probe.py): XXH64 batches of 4..64 buffers,
#      streaming XXH3, one-buffer XXH3 batch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03s2}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
use() { cp ab/lib$1.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so; }
X="--steps 12 --warmup 2 --batches 2 --coalesce 1 --timing-launches 8 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0"
use A &&
step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -2 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
TAG=$T/c2 REPS=3 bash scripts/ab_lib.sh python -u bench.py --steps 20 --warmup 5 --no-configs --e2e-batches 0 --no-cpu-baseline &&
TAG=$T/t16 REPS=2 bash scripts/ab_lib.sh python -u bench.py --buffers 16 --buffer-bytes 67108864 $X &&
step 60 $O/chainbench.json aws-crt-cpp_amd/build/tools/chainbench && cat $O/chainbench.json &&
use A && VARIANT=A step 300 $O/hash_probe_A.json python -u aws-crt-cpp_amd/tools/hash_probe.py && tail -1 $O/hash_probe_A.json &&
use C && VARIANT=C step 300 $O/hash_probe_C.json python -u aws-crt-cpp_amd/tools/hash_probe.py && tail -1 $O/hash_probe_C.json &&
use A && step 120 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && tail -1 $O/smoke.log &&
echo "session ok"
