#!/bin/bash
# XXH3 long-path variants: GPU parity suite, then C2-shape and 8 x 64 MiB XXH3-64 / XXH3-128.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-xxh3b}; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 150 python bench.py --no-cpu-baseline --e2e-batches 0 --target-buffers 0 "$@" > $O/$tag.log 2>&1 || return $?;
  grep '^{' $O/$tag.log | tail -1 > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); r=d['roofline']; print('%-14s' % '$tag', d['value'], 'GiB/s', d['pct_hbm_peak'], '% peak; kernel', r['kernel_ms'], 'frac', r['frac'])"; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && tail -1 $O/pytest.log &&
run c2_xxh3 --alg xxh3_64 --steps 100 --warmup 10 --timing-launches 8 &&
run c2_xxh3_128 --alg xxh3_128 --steps 100 --warmup 10 --timing-launches 8 &&
run c5_xxh3 --alg xxh3_64 --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 4 --warmup 1 --timing-launches 2 --no-read-ceiling
