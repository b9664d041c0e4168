#!/bin/bash
# Round-3 session 4.
#   ab3/libA.so = release candidate (crc64_rows16_kernel for short CRC64NVME buffers, XXH64 host
#   route up to 16 buffers); B = A without rows16; C = A with 1024-thread crc64_stream4 workgroups.
#   ab2/lib{A..E}.so = ragged-list experiments: B, C = list tiles of 1/2, 1/4 size; D = workgroup
#   tile pool for lists; E = pool + half-size tiles.
#   1. GPU parity suite on ab3/A; the list paths on ab2/B (the pool variants D, E failed parity:
#      test_ragged_list_random, session r03s4 first attempt; dropped)
#   2. C4 shard CRC64NVME A/B/C and C5 CRC64NVME A/C (config-leg shape: pipelined value + isolated kernel)
#   3. the list probe on ab2 A..E
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03s4}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
use() { cp $1.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so; }
K="list or multipart or ingest or fuzz or front_pad or eventstream"
X="--steps 12 --warmup 2 --batches 2 --coalesce 1 --timing-launches 8 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0"
P="--steps 12 --warmup 4 --batches 2 --coalesce 1 --timing-launches 8 --branches 3 --no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
use ab3/libA && step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
use ab2/libB && step 300 $O/pytest_listB.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" &&
tail -1 $O/pytest_listB.log && ! grep -q "failed" $O/pytest_listB.log &&
mkdir -p ab && cp ab3/*.so ab/ &&
VARIANTS="A B C" TAG=$T/c4 REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 131072 --buffer-bytes 8192 $X &&
VARIANTS="A C" TAG=$T/c5p REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 $P &&
LIBDIR=ab2 VARIANTS="A B C" TAG=$T/lists REPS=2 bash scripts/ab_listprobe.sh &&
cp ab3/libA.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so &&
echo "session ok"
