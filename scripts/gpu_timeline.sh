#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 120 python aws-crt-cpp_amd/tools/timeline.py --buffers 16 --buffer-bytes 67108864 --launches 5 &&
timeout -k 10 120 python aws-crt-cpp_amd/tools/timeline.py
