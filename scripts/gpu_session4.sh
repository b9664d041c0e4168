#!/bin/bash
# GPU session: smoke (any failure ends the session), gpu tests, bench shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
S=scripts/gpu_step.sh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
$S 900 $O/pytest_gpu.log python -m pytest tests -m gpu -q -p no:cacheprovider &&
$S 300 $O/bench_graph.log python bench.py --steps 400 --warmup 20 --cpu-seconds 5 &&
$S 300 $O/bench_4m.log python bench.py --steps 400 --warmup 20 --no-cpu-baseline --buffers 16 --buffer-bytes 4194304 &&
$S 300 $O/bench_64m.log python bench.py --steps 100 --warmup 10 --no-cpu-baseline --buffers 16 --buffer-bytes 67108864 --batches 2 &&
$S 300 $O/bench_crc32.log python bench.py --steps 400 --warmup 20 --no-cpu-baseline --alg crc32
echo "session rc=$?"
tail -3 $O/smoke.log; tail -15 $O/pytest_gpu.log
for f in bench_graph bench_4m bench_64m bench_crc32; do grep -h metric $O/$f.log | python3 -c "import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; print('$f', d['value'], d['unit'], 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'cpu', (d.get('cpu_baseline') or {}).get('value'))"; done
