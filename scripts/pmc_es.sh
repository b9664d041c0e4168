#!/bin/bash
# SQ / cache counter passes of the event-stream framing kernels, per library build ab/lib$v.so (v in
# $VARIANTS), swapped into aws-crt-cpp_amd/lib/ in turn (the release build is put back at the end).
# Outputs under gpurun_out/$TAG/<v>_<pass>.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${TAG:-pmces}; mkdir -p $O; export TMPDIR=/tmp
L=aws-crt-cpp_amd/lib/libaws-checksums-amd.so
cp $L /tmp/pmces_release.so
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
P2="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
rc=0
for v in ${VARIANTS:-C ESL}; do
  cp ab/lib$v.so $L || { rc=1; break; }
  for pass in P1 P2; do
    eval C=\$$pass
    (cd /tmp && timeout -s KILL 100 rocprofv3 --pmc $C -d $O/${v}_$pass -o run --output-format csv -- python3 $R/aws-crt-cpp_amd/tools/bench_eventstream.py --device-frames --steps 12 --timing-launches 4) > $O/${v}_$pass.log 2>&1 || { rc=$?; echo "pass $v $pass failed"; break 2; }
  done
done
cp /tmp/pmces_release.so $L
[ $rc -eq 0 ] && echo "pmces ok"
exit $rc
