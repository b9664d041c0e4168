#!/bin/bash
# Braided (list / unaligned) scans: GPU suite on ab/libB.so, then the list probe on A and B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-lists}; mkdir -p $O
# SKIP_TEST=1: timing-only variants (e.g. a build with work removed) skip the suite
if [ -z "${SKIP_TEST:-}" ]; then
  cp ab/libB.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so &&
  bash scripts/gpu_step.sh 600 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider &&
  tail -1 $O/pytest.log && grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log || exit 1
fi
for r in 1 2; do
  for v in A B; do
    cp ab/lib$v.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
    bash scripts/gpu_step.sh 120 $O/${v}_$r.log python -u aws-crt-cpp_amd/tools/list_probe.py ${PROBE_ARGS:-} || exit 1
    echo "$v $r $(grep '^{' $O/${v}_$r.log)"
  done
done
cp ab/lib${KEEP:-B}.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so
if [ -n "${BENCH_AB:-}" ]; then
  TAG=${TAG:-lists}/bench REPS=2 bash scripts/ab_lib.sh python -u bench.py $BENCH_AB
fi
