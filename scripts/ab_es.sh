#!/bin/bash
# A/B of event-stream builds on one box: ab/lib$v.so (v in ${VARIANTS}) swapped into aws-crt-cpp_amd/lib/
# alternately, tools/bench_eventstream.py --device-frames run against each, REPS times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-abes}; mkdir -p $O
cp aws-crt-cpp_amd/lib/libaws-checksums-amd.so /tmp/ab_release.so
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-A B}; do
    cp ab/lib$v.so aws-crt-cpp_amd/lib/libaws-checksums-amd.so || exit 1
    timeout -k 10 120 python aws-crt-cpp_amd/tools/bench_eventstream.py --device-frames ${ES_ARGS:---timing-only} > $O/${v}_$r.log 2>&1 || exit 1
    echo "$v $r $(grep '^{' $O/${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["kernel_ms"], d["roofline_frac"], d["value"])')"
  done
done
cp /tmp/ab_release.so aws-crt-cpp_amd/lib/libaws-checksums-amd.so
