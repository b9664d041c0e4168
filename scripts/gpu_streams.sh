#!/bin/bash
# C2 pipelined rate against the number of streams, paired and single-chain streaming scans.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-st}; mkdir -p $O
run() { local tag=$1; shift; local br=$1; shift; env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 --steps 400 --branches $br > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('%-22s' % '$tag', d['value'], 'GiB/s', 'kernel', d['roofline']['kernel_ms'])"; }
for br in 2 3 4 6; do
  run pair_b$br $br X=1 && run single512_b$br $br AMDCRC_DEBUG=8192 AMDCRC_SEG=512 || exit $?
done
run pair_b3_again 3 X=1 && run single512_b3_again 3 AMDCRC_DEBUG=8192 AMDCRC_SEG=512
