#!/bin/bash
# Round-3 session v20: the XXH64 host route on the host path's persistent workers (N) vs a thread per
# buffer per slice (A): XXH64 parity on N, then C5 XXH64 (8 x 64 MiB) through bench.py, 3 reps each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; T=${TAG:-r03v20}; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
cp ab/libN.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
bash scripts/gpu_step.sh 300 $O/pytest_x64.log python -u -m pytest tests/test_gpu_parity.py tests/test_streaming_xxhash.py -m gpu -x -q -k "xxh64 or XXH64 or host_route or C5 or c5" --timeout 120 --timeout-method thread -p no:cacheprovider &&
tail -1 $O/pytest_x64.log && grep -q " passed" $O/pytest_x64.log && ! grep -q "failed" $O/pytest_x64.log || exit 1
for r in 1 2 3; do for v in A N; do
  cp ab/lib$v.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so || exit 1
  bash scripts/gpu_step.sh 200 $O/${v}_$r.log python -u bench.py --alg xxh64 --buffers 8 --buffer-bytes 67108864 --batches 2 --steps 8 --warmup 2 --timing-launches 2 --no-configs --no-cpu-baseline --e2e-batches 0 --no-read-ceiling || exit 1
  echo "$v $r $(grep '^{' $O/${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done; done
cp ab/libN.so aws-crt-cpp_amd/lib/libaws-crt-cpp-amd.so
echo "session ok"
