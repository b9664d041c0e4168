#!/bin/bash
# Round-3 session v13: crc32_list_stream_kernel with cut parts held and published after the scan
# (A, in tree) vs the previous list kernel (P): the list parity tests and multipart / host-ingest
# tests on A, then the ragged-list probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v13}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
bash scripts/gpu_step.sh 400 $O/pytest_lists.log python -u -m pytest tests/test_gpu_parity.py tests/test_multipart.py tests/test_host_ingest.py -m gpu -x -q -k "list or ragged or multipart or ingest or host or fuzz or pad" --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest_lists.log && grep -q " passed" $O/pytest_lists.log && ! grep -q "failed" $O/pytest_lists.log &&
TAG=$T/lists VARIANTS="A P" REPS=3 LIBDIR=ab bash scripts/ab_listprobe.sh &&
echo "session ok"
