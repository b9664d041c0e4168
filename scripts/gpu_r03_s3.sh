#!/bin/bash
# Round-3 session 3 (ab/libA.so = the release build):
#   1. GPU parity suite on A
#   2. where the CRC64NVME streaming scan's time goes: A vs experiment builds B (no tile finish
#      product), C (address perms without the table reads), D (no per-lane dword select), E (one
#      1024-thread workgroup per CU) on C5 and the C4 shard (2 reps)
#   3. XXH64 batches on device data: A (double-buffered host route up to 24 buffers) vs F (GPU kernels)
#   4. the driver's bench command, plain and under a kernel trace, matched launch by launch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03s3}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
use() { cp ab/lib$1.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so; }
X="--steps 12 --warmup 2 --batches 2 --coalesce 1 --timing-launches 8 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0"
use A &&
step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -2 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
VARIANTS="A B C D E" TAG=$T/c5 REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 $X &&
VARIANTS="A B C D E" TAG=$T/c4 REPS=2 bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 131072 --buffer-bytes 8192 $X &&
use A && VARIANT=A step 300 $O/hash_probe_A.json python -u aws-crt-cpp_amd/tools/hash_probe.py --counts 4,8,16,20,24,28,32 && tail -1 $O/hash_probe_A.json &&
use F && VARIANT=F step 300 $O/hash_probe_F.json python -u aws-crt-cpp_amd/tools/hash_probe.py --counts 4,8,16,20,24,28,32 && tail -1 $O/hash_probe_F.json &&
use A && step 400 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 && grep '^{' $O/bench_driver.log | cut -c1-400 &&
(cd /tmp && step 420 $O/prof_driver.log rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5) &&
python3 aws-crt-cpp_amd/tools/trace_match.py $O/prof_driver/run_kernel_trace.csv $O/prof_driver.log > $O/trace_match.json && tail -5 $O/trace_match.json &&
echo "session ok"
