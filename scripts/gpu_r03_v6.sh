#!/bin/bash
# Round-3 session v6 (crc64_xcd_kernel in tree): full GPU suite, smoke, the driver's bench command and a
# kernel trace of it, then counter passes: C5 FETCH_SIZE and SQ on crc64_xcd_kernel, C2 SQ on the
# 20-batch crc32_stream_kernel launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v6}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
C2="--steps 20 --warmup 20 --only-coalesced --branches 1 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 16 --no-read-ceiling"
C5="--alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 12 --warmup 2 --timing-launches 6 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
step 180 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && tail -1 $O/smoke.log &&
step 400 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 && grep '^{' $O/bench_driver.log | cut -c1-300 &&
cd /tmp &&
step 420 $O/prof_driver.log rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 &&
pmc() { n=$1; c=$2; shift 2; step 120 $O/$n.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/$n -o run --output-format csv -- python3 $R/bench.py "$@"; }
pmc c5_fetch "FETCH_SIZE" $C5 &&
pmc c5_sqa "$SQA" $C5 &&
pmc c2_sqa "$SQA" $C2 &&
echo "session ok"
