#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
B=aws-crt-cpp_amd/build/tools/overlapbench
timeout -k 10 100 $B 1 64 2 > $O/ov_64_2.log 2>&1 &&
timeout -k 10 100 $B 1 1024 1 > $O/ov_1024_1.log 2>&1
rc=$?
cat $O/ov_64_2.log $O/ov_1024_1.log
exit $rc
