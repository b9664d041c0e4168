#!/bin/bash
# Round-3 session v10: crc32_stream_kernel tiles in XCD-window order for one-tile buffers.
# A = off (release), S = tiles <= 16 KiB (C4 shard), L = every one-tile batch (C2 too).
# 1. the full GPU parity suite on L; 2. config legs for A / S / L, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v10}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
cp ab/libL.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
bash scripts/gpu_step.sh 600 $O/pytest_L.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest_L.log && grep -q " passed" $O/pytest_L.log && ! grep -q "failed" $O/pytest_L.log || { cp ab/libA.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so; exit 1; }
VARIANTS="A S L" TAG=$T bash scripts/gpu_r03_v9.sh
