#!/bin/bash
# Round-2 validation on the restored tree: GPU suite, smoke, driver-shaped bench, and an A/B of the
# host's completion wait (HIP runtime default vs ROC_ACTIVE_WAIT_TIMEOUT spin) on the timed region.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${TAG:-r02v}; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
step 900 $O/pytest.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS:-} &&
tail -2 $O/pytest.log &&
step 200 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && tail -1 $O/smoke.log &&
step 120 $O/probe_default.log python -u aws-crt-cpp_amd/tools/overhead_probe.py 20 && tail -1 $O/probe_default.log &&
ROC_ACTIVE_WAIT_TIMEOUT=2000 step 120 $O/probe_spin.log python -u aws-crt-cpp_amd/tools/overhead_probe.py 20 && tail -1 $O/probe_spin.log &&
step 200 $O/bench20.log python -u bench.py --steps 20 --warmup 5 --no-configs --e2e-batches 0 --no-cpu-baseline && grep "^{" $O/bench20.log | cut -c1-200 &&
ROC_ACTIVE_WAIT_TIMEOUT=2000 step 200 $O/bench20_spin.log python -u bench.py --steps 20 --warmup 5 --no-configs --e2e-batches 0 --no-cpu-baseline && grep "^{" $O/bench20_spin.log | cut -c1-200 &&
step 200 $O/bench20_b.log python -u bench.py --steps 20 --warmup 5 --no-configs --e2e-batches 0 --no-cpu-baseline && grep "^{" $O/bench20_b.log | cut -c1-200 &&
ROC_ACTIVE_WAIT_TIMEOUT=2000 step 200 $O/bench20_spin_b.log python -u bench.py --steps 20 --warmup 5 --no-configs --e2e-batches 0 --no-cpu-baseline && grep "^{" $O/bench20_spin_b.log | cut -c1-200 &&
C5="--alg crc64nvme --steps 20 --warmup 2 --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --timing-launches 8 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0" &&
TAG=${TAG:-r02v}/ab_c5 REPS=2 bash scripts/ab_lib.sh python -u bench.py $C5 &&
B16="--alg crc64nvme --steps 8 --warmup 2 --buffers 65536 --buffer-bytes 16384 --batches 2 --coalesce 1 --timing-launches 8 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0" &&
TAG=${TAG:-r02v}/ab_b16 REPS=2 bash scripts/ab_lib.sh python -u bench.py $B16 &&
echo "session ok"
