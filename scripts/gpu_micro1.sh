#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
B=aws-crt-cpp_amd/build/tools/microbench
timeout -k 10 120 $B 64 256 200 8 > $O/micro_64_256.log 2>&1 &&
timeout -k 10 120 $B 64 128 200 8 > $O/micro_64_128.log 2>&1 &&
timeout -k 10 120 $B 64 64 200 8 > $O/micro_64_64.log 2>&1 &&
timeout -k 10 120 $B 1024 256 50 2 > $O/micro_1024_256.log 2>&1 &&
timeout -k 10 120 $B 1024 1024 50 2 > $O/micro_1024_1024.log 2>&1
echo "rc=$?"
grep -h "round 2" $O/micro_*.log
