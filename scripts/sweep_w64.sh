#!/bin/bash
# CRC64NVME vs CRC32C at equal launch shapes (C5 8 x 64 MiB, C2 1024 x 64 KiB), one and many batches per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-w64}; mkdir -p $O
B="--no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 8 --no-read-ceiling"
for alg in crc64nvme crc32c; do
  for shape in "--buffers 8 --buffer-bytes 67108864 --batches 2" "--buffers 1024 --buffer-bytes 65536 --batches 8"; do
    for g in 1 8; do
      f=$O/${alg}_$(echo $shape | awk '{print $2"x"$4}')_g$g.json
      timeout -k 10 120 python -u bench.py --alg $alg $shape --coalesce $g --steps 40 --warmup 8 $B > $f 2>$O/err.log || exit $?
      python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);r=d['roofline'];print(sys.argv[1].split('/')[-1],d['value'],r['frac'],r['kernel_ms'],r.get('single_batch',{}).get('frac'))" $f
    done
  done
done
