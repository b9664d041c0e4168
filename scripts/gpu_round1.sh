#!/bin/bash
# Round-1 GPU session: parity tests, smoke, headline bench, rocprofv3 kernel trace + HBM PMC passes.
# Every GPU step has its own time limit; the first fault-like exit ends the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r1}; mkdir -p $O
export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
B="--steps 200 --warmup 20"
P="--steps 16 --warmup 16 --timing-launches 8 --no-cpu-baseline --e2e-batches 0 --target-buffers 0"

step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -3 $O/pytest.log &&
step 180 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" &&
tail -2 $O/smoke.log &&
step 240 $O/bench.log python -u bench.py $B &&
tail -1 $O/bench.log &&
step 120 $O/timeline.log python aws-crt-cpp_amd/tools/timeline.py &&
head -12 $O/timeline.log &&
cd /tmp &&
step 240 $O/prof.log rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 0 --warmup 0 --no-cpu-baseline --e2e-batches 0 --target-buffers 0 &&
step 120 $O/pmc_fetch.log rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py $P &&
step 120 $O/pmc_rdreq.log rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/pmc_rdreq -o run --output-format csv -- python3 $R/bench.py $P
echo "session rc=$?"
cd $R
find $O -name '*.csv' | head -20
