#!/bin/bash
# Launch-shape experiments for the C2 headline: graph vs eager, branch count, batch size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/exp1; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
run g1 --branches 1 &&
run g2 --branches 2 &&
run g4 --branches 4 &&
run e1 --mode eager --branches 1 &&
run e2 --mode eager --branches 2 &&
run big --buffers 16 --buffer-bytes 67108864 --batches 2 --steps 40 --warmup 4 --timing-launches 8 &&
run big256 --buffers 4096 --buffer-bytes 65536 --batches 2 --steps 40 --warmup 4 --timing-launches 8 &&
timeout -k 10 120 python aws-crt-cpp_amd/tools/timeline.py --buffers 16384 > $O/tl_1g.log 2>&1 && head -9 $O/tl_1g.log
