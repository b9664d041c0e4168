#!/bin/bash
# A/B of library builds ($LIBDIR/lib$v.so, v in ${VARIANTS:-A B}) on the ragged-list probe
# (aws-crt-cpp_amd/tools/list_probe.py ${ALG:-crc32c}), REPS times; one JSON line per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-abl}; mkdir -p $O; D=${LIBDIR:-ab}
cp aws-crt-cpp_amd/lib/libaws-checksums-amd.so /tmp/ab_release.so  # put back at the end
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-A B}; do
    cp $D/lib$v.so aws-crt-cpp_amd/lib/libaws-checksums-amd.so || exit 1
    bash scripts/gpu_step.sh 200 $O/${v}_$r.json python -u aws-crt-cpp_amd/tools/list_probe.py ${ALG:-crc32c} || exit 1
    echo "$v $r $(grep '^{' $O/${v}_$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print({k: v for k, v in d.items() if not k.endswith("_gibs") and k != "list_ragged_bytes"})')"
  done
done
cp /tmp/ab_release.so aws-crt-cpp_amd/lib/libaws-checksums-amd.so
