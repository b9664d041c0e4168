#!/bin/bash
# A/B of library builds (ab/lib$v.so, v in $VARIANTS) on the driver-shaped timed region: the overhead
# probe's median wall time of one synchronised 20-batch launch (30 repetitions), REPS times each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-abp}; mkdir -p $O
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-A B}; do
    cp ab/lib$v.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
    bash scripts/gpu_step.sh 120 $O/${v}_$r.log python -u aws-crt-cpp_amd/tools/overhead_probe.py ${NBATCH:-20} || exit 1
    echo "$v $r $(grep '^{' $O/${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline())["c2_'${NBATCH:-20}'_batches"]; print(d["wall_us"], d["kernel_us"], d["marker_to_marker_us"])')"
  done
done
cp ab/libA.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so
