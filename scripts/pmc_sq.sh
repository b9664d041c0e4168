#!/bin/bash
# SQ issue/stall breakdown of the C5 CRC64NVME launch and of the CRC32C target-shape launch (one
# counter pass each, 8 SQ counters + GRBM_GUI_ACTIVE).  Outputs under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${TAG:-sq}; mkdir -p $O; export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
B="--steps 6 --warmup 2 --batches 2 --coalesce 1 --timing-launches 4 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0"
cd /tmp
for w in "c5 --alg crc64nvme --buffers 8 --buffer-bytes 67108864" "t16 --alg crc32c --buffers 16 --buffer-bytes 67108864" ${EXTRA:+"$EXTRA"}; do
  set -- $w; n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc $C -d $O/$n -o run --output-format csv -- python3 $R/bench.py $B "$@" > $O/$n.log 2>&1 || { echo "pass $n failed"; exit 1; }
done
echo "sq ok"
