#!/bin/bash
# Round-3 session v25: tree with crc64_list_stream_kernel for padded CRC64NVME lists (A; unpadded lists
# stay on crc64_braid_kernel<LIST>) vs the previous tree (P): full GPU suite and smoke on A, the list
# probe A / P, a rocprof kernel trace of the CRC64 list probe on A, the driver's bench command on A.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v25}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
cp ab/libA.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
step 180 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && tail -1 $O/smoke.log &&
TAG=$T/probe VARIANTS="A P" REPS=2 ALG=crc64nvme bash scripts/ab_listprobe.sh &&
cd /tmp &&
step 300 $O/prof_list64.log rocprofv3 --kernel-trace --stats -d $O/prof_list64 -o run --output-format csv -- python3 $R/aws-crt-cpp_amd/tools/list_probe.py crc64nvme &&
cd $R &&
step 400 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 && grep '^{' $O/bench_driver.log | cut -c1-300 &&
echo "session ok"
