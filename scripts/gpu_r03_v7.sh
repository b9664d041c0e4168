#!/bin/bash
# Round-3 session v7: the box's counter list, then instruction-fetch and scalar-instruction counters
# on the 20-batch C2 launch (crc32_stream_kernel) and on C5 (crc64_xcd_kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v7}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
C2="--steps 20 --warmup 20 --only-coalesced --branches 1 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 16 --no-read-ceiling"
C5="--alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 12 --warmup 2 --timing-launches 6 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling"
cd /tmp
step 90 $O/counters.txt timeout -s KILL 60 rocprofv3 -L
grep -oE "(SQC|SQ)_[A-Z0-9_]+" $O/counters.txt | sort -u > $O/sq_names.txt
pmc() { n=$1; c=$2; shift 2; step 120 $O/$n.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/$n -o run --output-format csv -- python3 $R/bench.py "$@"; }
pmc c2_ic "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE" $C2 &&
pmc c5_ic "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE" $C5 &&
echo "session ok"
