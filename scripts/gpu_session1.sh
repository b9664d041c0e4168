#!/bin/bash
# First GPU session: smoke, gpu parity tests, short bench, rocprof kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" &&
$S 900 $O/pytest_gpu.log python -m pytest tests -m gpu -q -x -p no:cacheprovider &&
$S 300 $O/bench.log python bench.py --steps 200 --warmup 20 --cpu-seconds 5 &&
$S 300 $O/rocprof.log rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline
echo "session rc=$?"
tail -3 $O/smoke.log; tail -15 $O/pytest_gpu.log; cat $O/bench.log | tail -3
