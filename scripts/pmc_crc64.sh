#!/bin/bash
# Counter passes over tools/crc64_probe.py (CRC64NVME vs CRC32C vs read ceiling, C5 one-batch and
# 20-batch launches, C4 shard): VERDICT r05 item 3.  One rocprofv3 --pmc pass per counter set, each
# under its own kill timer.  Outputs under gpurun_out/$TAG/<set>.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${TAG:-pmc64}; mkdir -p $O; export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
cd /tmp
for set in A B; do
  eval C=\$$set
  timeout -s KILL 150 rocprofv3 --pmc $C -d $O/$set -o run --output-format csv -- python3 $R/aws-crt-cpp_amd/tools/crc64_probe.py --reps 1 --launches 4 > $O/$set.log 2>&1 || { echo "pass $set failed"; tail -5 $O/$set.log; exit 1; }
done
echo "pmc64 ok"
