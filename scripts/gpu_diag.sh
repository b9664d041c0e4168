#!/bin/bash
# Decompose the C2 launch: single-chain streaming scan with parts disabled (AMDCRC_DEBUG DIAG bits;
# results are wrong by construction, so the bench's parity flag is ignored here).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-dg}; mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 --steps 300 ${BARGS} > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('%-22s' % '$tag', d['value'], 'GiB/s', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
run single AMDCRC_DEBUG=8192 AMDCRC_SEG=512 &&
run notables AMDCRC_DEBUG=$((8192 + 65536)) AMDCRC_SEG=512 &&
run nofinish AMDCRC_DEBUG=$((8192 + 131072)) AMDCRC_SEG=512 &&
run nolookup AMDCRC_DEBUG=$((8192 + 262144)) AMDCRC_SEG=512 &&
run readonly AMDCRC_DEBUG=$((8192 + 458752)) AMDCRC_SEG=512 &&
run pair X=1 &&
run single256 AMDCRC_DEBUG=8192
