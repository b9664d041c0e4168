#!/bin/bash
# Round-3 evidence session on the shipped kernels (no code change): the counter list of this box,
# SQ issue/stall passes and a FETCH_SIZE pass on the 20-batch C2 launch (crc32_stream_kernel) and on
# C5 (crc64_stream4_kernel), then a kernel trace of the driver's exact bench command, so every
# config leg's event timing can be matched with rocprof's durations of the same dispatches.
# Outputs under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${TAG:-r03ev}; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
C2="--steps 20 --warmup 20 --only-coalesced --branches 1 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 16"
C5="--alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 12 --warmup 2 --timing-launches 6 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0"
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
SQB="SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
cd /tmp
(timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true)
pmc() { n=$1; c=$2; shift 2; step 120 $O/$n.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/$n -o run --output-format csv -- python3 $R/bench.py "$@"; }
pmc c2_sqa "$SQA" $C2 &&
pmc c5_sqa "$SQA" $C5 &&
pmc c5_fetch "FETCH_SIZE" $C5 &&
step 420 $O/prof_driver.log rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 &&
pmc c2_sqb "$SQB" $C2 &&
echo "evidence ok"
