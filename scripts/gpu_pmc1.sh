#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O/pmc1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > $O/pmc1/counters.txt 2>&1
grep -oE "^(SQ|TCC|TCP|GRBM|TA|TD)[A-Z0-9_]*" $O/pmc1/counters.txt | sort -u > $O/pmc1/names.txt
wc -l $O/pmc1/names.txt
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM"
G="--buffers 16 --buffer-bytes 67108864 --batches 2 --steps 6 --warmup 2 --no-cpu-baseline --timing-launches 4"
timeout -k 10 300 rocprofv3 --pmc $C -d $O/pmc1/bench -o run --output-format csv -- python3 bench.py $G > $O/pmc1/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc $C -d $O/pmc1/micro -o run --output-format csv -- aws-crt-cpp_amd/build/tools/overlapbench 1 1024 1 > $O/pmc1/micro.log 2>&1
echo rc=$?
