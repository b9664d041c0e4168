#!/bin/bash
# A/B of checksum-library builds on any command: ab/lib$v.so (v in ${VARIANTS:-A B}) swapped into
# aws-crt-cpp_amd/lib/libaws-checksums-amd.so alternately, the command run against each, REPS times;
# logs under gpurun_out/$TAG/<v>_<rep>.log.  The release build is put back at the end.
#   VARIANTS="R NX" REPS=2 bash scripts/ab_cmd.sh python -u aws-crt-cpp_amd/tools/crc64_probe.py --only c5_20
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-abc}; mkdir -p $O
L=aws-crt-cpp_amd/lib/libaws-checksums-amd.so
cp $L /tmp/ab_release.so
rc=0
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-A B}; do
    cp ab/lib$v.so $L || { rc=1; break 2; }
    bash scripts/gpu_step.sh ${STEP_TIMEOUT:-200} $O/${v}_$r.log "$@" || { rc=$?; break 2; }
    echo "$v $r"; grep '^{' $O/${v}_$r.log | cut -c1-300
  done
done
cp /tmp/ab_release.so $L
exit $rc
