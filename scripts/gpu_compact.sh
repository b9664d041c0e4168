#!/bin/bash
# Compact-table CRC32C streaming scan (AMDCRC_DEBUG bit 21, 46 KiB LDS, 3 workgroups per CU):
# parity, then C2/C3/C4 against the default kernel at 3-5 streams.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-cmp}; mkdir -p $O
AMDCRC_DEBUG=2097152 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "crc32c and (config2 or fuzz_strided or strided_shapes or config3 or config4)" > $O/pytestc.log 2>&1
rc=$?; tail -1 $O/pytestc.log; [ $rc -eq 0 ] || exit $rc
run() { local tag=$1; local ev=$2; shift 2; env $ev timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-batches 0 --no-read-ceiling "$@" > $O/$tag.log 2>&1 || return $?;
  tail -1 $O/$tag.log > $O/$tag.json; python3 -c "import json; d=json.load(open('$O/$tag.json')); print('%-22s' % '$tag', d['value'], 'GiB/s', 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
run c2_def_b3 X=1 --steps 400 &&
run c2_cmp_b3 AMDCRC_DEBUG=2097152 --steps 400 &&
run c2_cmp_b4 AMDCRC_DEBUG=2097152 --steps 400 --branches 4 &&
run c2_cmp_b2 AMDCRC_DEBUG=2097152 --steps 400 --branches 2 &&
run c2_cmp_b6 AMDCRC_DEBUG=2097152 --steps 400 --branches 6 &&
run c2_def_b3_again X=1 --steps 400 &&
run c2_cmp_b3_again AMDCRC_DEBUG=2097152 --steps 400
