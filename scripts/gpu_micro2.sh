#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
B=aws-crt-cpp_amd/build/tools/microbench2
timeout -k 10 200 $B 64 200 8 > $O/micro2_64.log 2>&1 &&
timeout -k 10 200 $B 1024 30 2 > $O/micro2_1024.log 2>&1
echo "rc=$?"
grep -h "round 1" $O/micro2_64.log $O/micro2_1024.log
