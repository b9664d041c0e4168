#!/bin/bash
# Round-3 session v9: config legs (warmed streams, 3-stream pipelines) for A (in tree) vs Z
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v9}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do for v in ${VARIANTS:-A Z}; do
  cp ab/lib$v.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
  bash scripts/gpu_step.sh 300 $O/${v}_$r.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-batches 0 --no-read-ceiling || exit 1
  grep '^{' $O/${v}_$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.readline())
print('$v $r', 'C2', d['value'], d['roofline']['kernel_ms'], *[(k, v['value'], v['roofline']['kernel_ms']) for k, v in d['configs'].items() if 'xxh' not in k])"
done; done
cp ab/libA.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so
echo "session ok"
