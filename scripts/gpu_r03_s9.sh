#!/bin/bash
# Round-3 session 9: the group-balanced list streaming scan (in-tree = ab/libA.so)
#   1. the full GPU parity suite
#   2. ragged-list probe: A vs T (tile-based list streaming scan, session 8) vs C (round-2 list kernel)
#   3. a kernel trace of A's probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03s9}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
TAG=$T/lists VARIANTS="A T C" REPS=2 LIBDIR=ab bash scripts/ab_listprobe.sh &&
(cd /tmp && step 200 $O/prof_lists.log rocprofv3 --kernel-trace --stats -d $O/prof_lists -o run --output-format csv -- python3 $R/aws-crt-cpp_amd/tools/list_probe.py crc32c) &&
echo "session ok"
