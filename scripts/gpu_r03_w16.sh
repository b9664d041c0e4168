#!/bin/bash
# Round-3 session: the 16-byte-word CRC32 streaming scan (ab/libB.so; ab/libA.so = the same tree with
# AMDCRC_STREAM_W16=0, i.e. the round-2 8-byte-word kernel for every launch).
#   1. GPU parity suite on B (the W16 kernel serves every W=32 strided launch of >= 256 MiB)
#   2. A/B on one box: the driver-shaped C2 run (3 reps), C3 and the target shape (2 reps)
#   3. evidence: SQ issue/stall passes of the 20-batch C2 launch for A and B, FETCH_SIZE for B;
#      SQ + FETCH_SIZE on C5 (crc64_stream4_kernel); a kernel trace of the driver's bench command on B
# Outputs under gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03w16}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
use() { cp ab/lib$1.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so; }
C2="--steps 20 --warmup 20 --only-coalesced --branches 1 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 16"
C5="--alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 12 --warmup 2 --timing-launches 6 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0"
X="--steps 12 --warmup 2 --batches 2 --coalesce 1 --timing-launches 8 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0"
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
pmc() { n=$1; c=$2; shift 2; (cd /tmp && step 120 $O/$n.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/$n -o run --output-format csv -- python3 $R/bench.py "$@"); }
use B &&
step 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -2 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log &&
TAG=$T/c2 REPS=3 bash scripts/ab_lib.sh python -u bench.py --steps 20 --warmup 5 --no-configs --e2e-batches 0 --no-cpu-baseline &&
TAG=$T/c3 REPS=2 bash scripts/ab_lib.sh python -u bench.py --buffers 16 --buffer-bytes 268435456 $X &&
TAG=$T/t16 REPS=2 bash scripts/ab_lib.sh python -u bench.py --buffers 16 --buffer-bytes 67108864 $X &&
use B && pmc c2_sqa_B "$SQA" $C2 && pmc c2_fetch_B FETCH_SIZE $C2 &&
use A && pmc c2_sqa_A "$SQA" $C2 &&
use B && pmc c5_sqa "$SQA" $C5 && pmc c5_fetch FETCH_SIZE $C5 &&
(cd /tmp && step 420 $O/prof_driver.log rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5) &&
echo "session ok"
