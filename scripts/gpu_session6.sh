#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
run() { echo "== $*"; timeout -k 10 150 "$@" 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_multipart.py -q -x -p no:cacheprovider > $O/parity6.log 2>&1; rc=$?; tail -2 $O/parity6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python aws-crt-cpp_amd/tools/timeline.py > $O/tl6.log 2>&1 && head -9 $O/tl6.log &&
run python bench.py --steps 400 --no-cpu-baseline &&
run python bench.py --buffers 16 --buffer-bytes 67108864 --batches 2 --steps 60 --warmup 5 --no-cpu-baseline --timing-launches 16
