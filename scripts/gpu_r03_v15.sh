#!/bin/bash
# Round-3 session v15: VMEM / LDS latency counters (SQ_INST_LEVEL_* over SQ_INSTS_*) for the 20-batch
# C2 scan and the read-ceiling kernel of the same size (bench.py's read-ceiling legs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v15}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
C2="--steps 20 --warmup 5 --branches 1 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 8"
cd /tmp
pmc() { n=$1; c=$2; shift 2; step 150 $O/$n.log timeout -s KILL 130 rocprofv3 --pmc $c -d $O/$n -o run --output-format csv -- python3 $R/bench.py "$@"; }
pmc lat "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" $C2 &&
pmc lat2 "SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" $C2 &&
echo "session ok"
