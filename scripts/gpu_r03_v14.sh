#!/bin/bash
# Round-3 session v14: event-stream framing with length-sorted lanes (A, in tree) vs the previous
# kernel (P): the event-stream parity tests on A, then bench_eventstream --device-frames for both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v14}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
bash scripts/gpu_step.sh 300 $O/pytest_es.log python -u -m pytest tests/test_eventstream.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest_es.log && grep -q " passed" $O/pytest_es.log && ! grep -q "failed" $O/pytest_es.log &&
for r in 1 2; do for v in A P; do
  cp ab/lib$v.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
  bash scripts/gpu_step.sh 200 $O/${v}_$r.json python -u aws-crt-cpp_amd/tools/bench_eventstream.py --device-frames || exit 1
  echo "$v $r $(grep '^{' $O/${v}_$r.json | cut -c1-400)"
done; done
cp ab/libA.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so
echo "session ok"
