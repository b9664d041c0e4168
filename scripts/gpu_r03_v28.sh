#!/bin/bash
# Round-3 session v28 (final tree): full GPU suite, smoke, the driver's bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v28}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
step 180 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && tail -1 $O/smoke.log &&
step 400 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 && grep '^{' $O/bench_driver.log | cut -c1-300 &&
echo "session ok"
