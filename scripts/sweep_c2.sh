#!/bin/bash
# C2 launch-shape sweep: batches per launch x streams, at the driver's 20 steps and at 200 steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-sweep}; mkdir -p $O
for steps in 20 200; do
  for g in 1 4 8 16; do
    for br in 1 3; do
      timeout -k 10 120 python -u bench.py --steps $steps --warmup 5 --coalesce $g --branches $br --no-configs \
        --no-cpu-baseline --e2e-batches 0 --timing-launches 16 > $O/c2_s${steps}_g${g}_b${br}.json 2>$O/err.log || exit $?
      python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[1],d['value'],r['frac'],r['kernel_ms'],r['single_batch'])" $O/c2_s${steps}_g${g}_b${br}.json
    done
  done
done
