#!/bin/bash
# Round-2 measurement session: full GPU suite, default bench, driver-shaped bench, rocprofv3 kernel
# traces (headline coalesced launches, C3 and target shapes) and the FETCH_SIZE traffic pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${TAG:-r02c}; mkdir -p $O; export TMPDIR=/tmp
step() { bash $R/scripts/gpu_step.sh "$@"; }
PROF="--only-coalesced --branches 1 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 16"
step 900 $O/pytest.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS:-} &&
tail -2 $O/pytest.log &&
step 200 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && tail -1 $O/smoke.log &&
step 400 $O/bench.log python -u bench.py && grep '^{' $O/bench.log | cut -c1-300 &&
step 200 $O/bench20.log python -u bench.py --steps 20 --warmup 5 --no-configs && grep "^{" $O/bench20.log | cut -c1-300 &&
step 200 $O/bench20b.log python -u bench.py --steps 20 --warmup 5 --no-configs --e2e-batches 0 --no-cpu-baseline && grep "^{" $O/bench20b.log | cut -c1-300 &&
cd /tmp &&
step 300 $O/prof_c2.log rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 20 $PROF &&
step 300 $O/prof_c3.log rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 $R/bench.py --steps 12 --warmup 2 --buffers 16 --buffer-bytes 268435456 --batches 2 --coalesce 1 --timing-launches 6 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0 &&
step 300 $O/prof_t16.log rocprofv3 --kernel-trace --stats -d $O/prof_t16 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --buffers 16 --buffer-bytes 67108864 --batches 2 --coalesce 1 --timing-launches 6 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0 &&
step 300 $O/prof_c5.log rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --alg crc64nvme --steps 20 --warmup 2 --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --timing-launches 6 --branches 1 --only-coalesced --no-configs --no-cpu-baseline --e2e-batches 0 &&
step 120 $O/pmc_fetch.log timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 20 $PROF &&
echo "session ok"
