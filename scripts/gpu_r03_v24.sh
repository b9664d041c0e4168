#!/bin/bash
# Round-3 session v24: ragged CRC64NVME lists on crc64_list_stream_kernel (A) vs crc64_braid_kernel<LIST>
# (P, -DAMDCRC_LIST_STREAM64=0): CRC64 list / multipart / host-ingest parity on A, then the list probe A / P.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v24}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
cp ab/libA.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
bash scripts/gpu_step.sh 300 $O/pytest_A.log python -u -m pytest tests/test_gpu_parity.py tests/test_multipart.py tests/test_host_ingest.py -m gpu -x -q -k "crc64nvme or list_devices or multipart_no" --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest_A.log && grep -q " passed" $O/pytest_A.log && ! grep -q "failed" $O/pytest_A.log || exit 1
TAG=$T/probe VARIANTS="A P" REPS=2 ALG=crc64nvme bash scripts/ab_listprobe.sh &&
echo "session ok"
