#!/bin/bash
# One GPU session on the pool's box: the named steps in order, each under its own time limit; the
# first fault-like exit (abort, segv, timeout) ends the session.
#   TAG=r02a scripts/gpu_session.sh test smoke bench prof pmc
# Outputs under gpurun_out/$TAG (copy what is to be kept into profiles/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${TAG:-run}; mkdir -p $O
export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
# profiling runs: driver-shaped launches only (20 batches per launch), no CPU baseline or extra legs
P="--steps 20 --warmup 20 --only-coalesced --branches 1 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 16"
rc=0
for s in "$@"; do
  case $s in
    test)  step 900 $O/pytest.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider; rc=$?; tail -3 $O/pytest.log ;;
    smoke) step 180 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; tail -2 $O/smoke.log ;;
    bench) step 400 $O/bench.log python -u bench.py ${BENCH_ARGS:-}; rc=$?; tail -1 $O/bench.log ;;
    prof)  (cd /tmp && step 300 $O/prof.log rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py $P ${PROF_ARGS:-}); rc=$? ;;
    pmc)   (cd /tmp && step 120 $O/pmc_fetch.log timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py $P ${PROF_ARGS:-}); rc=$? ;;
    py:*)  n=$(basename ${s#py:} .py); step 600 $O/$n.log python -u ${s#py:}; rc=$?; tail -5 $O/$n.log ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  [ $rc -ne 0 ] && { echo "session stopped at $s rc=$rc"; exit $rc; }
done
echo "session ok"
