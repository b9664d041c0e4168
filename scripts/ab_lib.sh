#!/bin/bash
# A/B of builds of the library on one box: ab/lib$v.so (v in ${VARIANTS:-A B}) are swapped into
# aws-crt-cpp_amd/lib/ alternately and the same bench command runs against each, REPS times.
#   REPS=3 bash scripts/ab_lib.sh python -u bench.py --steps 20 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}; mkdir -p $O
cp aws-crt-cpp_amd/lib/libaws-checksums-amd.so /tmp/ab_release.so  # put back at the end
for r in $(seq 1 ${REPS:-3}); do
  for v in ${VARIANTS:-A B}; do
    cp ab/lib$v.so aws-crt-cpp_amd/lib/libaws-checksums-amd.so || exit 1
    bash scripts/gpu_step.sh 200 $O/${v}_$r.log "$@" || exit 1
    echo "$v $r $(grep '^{' $O/${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; sb=r.get("single_batch") or {}; print(d["value"], r["frac"], r["kernel_ms"], "one", (d.get("one_batch_per_launch") or {}).get("value"), "sb", sb.get("frac"), sb.get("kernel_ms"))')"
  done
done
cp /tmp/ab_release.so aws-crt-cpp_amd/lib/libaws-checksums-amd.so
