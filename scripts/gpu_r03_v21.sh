#!/bin/bash
# Round-3 session v21: the submission queue (aws_crt_amd_queue_*): full GPU suite (with tests/test_queue.py),
# then the driver's bench command (its queued_one_at_a_time leg).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v21}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
step 400 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-configs && grep '^{' $O/bench_driver.log | cut -c1-300 &&
echo "session ok"
