#!/bin/bash
# Round-3 session v18: head / tail bytes folded bit by bit on the scalar unit (N) vs through the LDS
# byte table (A): the full GPU suite on N, then the ragged-list probe A / N.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v18}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
cp ab/libN.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
bash scripts/gpu_step.sh 600 $O/pytest_N.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest_N.log && grep -q " passed" $O/pytest_N.log && ! grep -q "failed" $O/pytest_N.log || exit 1
TAG=$T/lists VARIANTS="A N" REPS=3 LIBDIR=ab bash scripts/ab_listprobe.sh &&
cp ab/libN.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so &&
echo "session ok"
