#!/bin/bash
# Round-3 session 5 on the release build (the in-tree library):
#   1. GPU parity suite and smoke
#   2. the driver's bench command twice and the default bench once
#   3. the driver's command under a kernel trace, matched launch by launch with its own events
#   4. FETCH_SIZE of the C4-shard CRC64NVME launch (crc64_rows16_kernel) and an SQ pass of it
#   5. where a 20-batch timed region's fixed time goes, with the default and the spinning host wait
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03s5}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
C4="--alg crc64nvme --buffers 131072 --buffer-bytes 8192 --batches 2 --coalesce 1 --steps 12 --warmup 2 --timing-launches 6 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0"
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
pmc() { n=$1; c=$2; shift 2; (cd /tmp && step 120 $O/$n.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/$n -o run --output-format csv -- python3 $R/bench.py "$@"); }
step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
step 120 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && tail -1 $O/smoke.log &&
step 400 $O/bench_driver_1.log python -u bench.py --gpus 1 --steps 20 --warmup 5 && grep '^{' $O/bench_driver_1.log | cut -c1-300 &&
step 400 $O/bench_driver_2.log python -u bench.py --gpus 1 --steps 20 --warmup 5 && grep '^{' $O/bench_driver_2.log | cut -c1-300 &&
step 500 $O/bench_default.log python -u bench.py && grep '^{' $O/bench_default.log | cut -c1-300 &&
(cd /tmp && step 420 $O/prof_driver.log rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5) &&
python3 aws-crt-cpp_amd/tools/trace_match.py $O/prof_driver/run_kernel_trace.csv $O/prof_driver.log > $O/trace_match.json &&
pmc c4_fetch FETCH_SIZE $C4 && pmc c4_sqa "$SQA" $C4 &&
step 120 $O/overhead_default.log python -u aws-crt-cpp_amd/tools/overhead_probe.py 20 && tail -1 $O/overhead_default.log &&
AMDCRC_PROBE_SCHED=spin step 120 $O/overhead_spin.log python -u aws-crt-cpp_amd/tools/overhead_probe.py 20 && tail -1 $O/overhead_spin.log &&
echo "session ok"
