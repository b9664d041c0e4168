#!/bin/bash
# Event-stream framing check, 16 lanes per message (ab/libB.so) vs one lane per message (ab/libA.so):
# the event-stream GPU tests on B, then bench_eventstream.py --device-frames on both, REPS times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-es}; mkdir -p $O
cp ab/libB.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so &&
bash scripts/gpu_step.sh 300 $O/pytest.log python -u -m pytest tests/test_eventstream.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest.log && ! grep -q "failed\|error" $O/pytest.log || exit 1
for r in $(seq 1 ${REPS:-2}); do
  for v in A B; do
    cp ab/lib$v.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
    bash scripts/gpu_step.sh 200 $O/${v}_$r.log python -u aws-crt-cpp_amd/tools/bench_eventstream.py --device-frames ${ES_ARGS:-} || exit 1
    echo "$v $r $(grep '^{' $O/${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["kernel_ms"], d["roofline_frac"])')"
  done
done
cp ab/libB.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so
