#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=aws-crt-cpp_amd/build/tools/overlapbench
timeout -k 10 100 $B 1 1024 1 | grep -E "dword" &&
timeout -k 10 100 $B 1 64 2 | grep -E "dword"
