#!/bin/bash
# Run one GPU step under its own time limit; stop the whole GPU session on a fault-like exit.
# usage: scripts/gpu_step.sh <seconds> <logfile> <cmd...>
# exit codes 0/1 (pass / ordinary test failure) let the caller continue; anything else (abort 134,
# segv 139, timeout 124/137, ...) is propagated so the caller stops using the GPU.
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc cmd=$*" >> "$log"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then exit 0; fi
echo "[gpu_step] FATAL rc=$rc in: $*" >&2
exit $rc
