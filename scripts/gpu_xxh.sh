#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/xxh; mkdir -p $O
timeout -k 10 300 python -m pytest -q -x tests/test_gpu_parity.py tests/test_cpp_dropin.py -p no:cacheprovider > $O/parity.log 2>&1; rc=$?; tail -3 $O/parity.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; shift; timeout -k 10 180 python bench.py --no-cpu-baseline --e2e-batches 0 "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], 'GiB/s', d['ms_per_step'], 'ms/step', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
run c2_xxh64 --alg xxh64 --steps 40 --warmup 4 --timing-launches 8 &&
run c2_xxh3 --alg xxh3_64 --steps 40 --warmup 4 --timing-launches 8 &&
run c2_xxh3_128 --alg xxh3_128 --steps 40 --warmup 4 --timing-launches 8 &&
run c5_xxh3 --alg xxh3_64 --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 6 --warmup 2 --timing-launches 2 --branches 2 &&
run c5_xxh64 --alg xxh64 --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 6 --warmup 2 --timing-launches 2 --branches 2 &&
run c5b_xxh64 --alg xxh64 --buffers 64 --buffer-bytes 67108864 --batches 1 --steps 4 --warmup 3 --timing-launches 2
