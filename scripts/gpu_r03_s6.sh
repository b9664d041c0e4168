#!/bin/bash
# Round-3 session 6: the list streaming scan (crc32_list_stream_kernel, ab/libA.so = the in-tree build)
#   1. list-related GPU parity tests on the new kernel
#   2. the ragged-list probe: A (list stream) / B (round-2 list kernel) / C (list stream, 2 tiles per slot)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03s6}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
step 300 $O/pytest_lists.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "list or multipart or ingest or fuzz or front_pad or devices or cpp_dropin" &&
tail -1 $O/pytest_lists.log && grep -q " passed" $O/pytest_lists.log && ! grep -q "failed" $O/pytest_lists.log &&
TAG=$T/lists VARIANTS="${VARIANTS:-A B C}" REPS=2 LIBDIR=ab bash scripts/ab_listprobe.sh &&
echo "session ok"
