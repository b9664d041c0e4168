#!/bin/bash
# GPU session: smoke (any failure ends the session), gpu tests, bench variants, rocprof trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
S=scripts/gpu_step.sh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
$S 900 $O/pytest_gpu.log python -m pytest tests -m gpu -q -p no:cacheprovider &&
$S 300 $O/bench_graph.log python bench.py --steps 400 --warmup 20 --cpu-seconds 5 &&
$S 300 $O/bench_graph1.log python bench.py --steps 400 --warmup 20 --branches 1 --no-cpu-baseline &&
$S 300 $O/bench_eager.log python bench.py --steps 400 --warmup 20 --mode eager --no-cpu-baseline &&
$S 300 $O/rocprof.log rocprofv3 --kernel-trace --stats -d $O/prof3 -o run --output-format csv -- python3 bench.py --steps 64 --warmup 8 --no-cpu-baseline
echo "session rc=$?"
tail -2 $O/smoke.log; tail -30 $O/pytest_gpu.log; for f in bench_graph bench_graph1 bench_eager; do grep -h metric $O/$f.log | cut -c1-600; done
