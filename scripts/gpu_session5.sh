#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_multipart.py -q -x -p no:cacheprovider > $O/multipart.log 2>&1; rc=$?
tail -3 $O/multipart.log
[ $rc -le 1 ] && bash scripts/gpu_timeline.sh
