#!/bin/bash
# Round-3 session 8: ragged-list probe, A (list streaming scan, in-tree) vs C (round-2 list kernel) vs
# D (2 tiles per wave slot) vs E (one workgroup per CU), then a kernel trace of A's probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03s8}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
TAG=$T/lists VARIANTS="A C D E" REPS=2 LIBDIR=ab bash scripts/ab_listprobe.sh &&
(cd /tmp && step 200 $O/prof_lists.log rocprofv3 --kernel-trace --stats -d $O/prof_lists -o run --output-format csv -- python3 $R/aws-crt-cpp_amd/tools/list_probe.py crc32c) &&
echo "session ok"
