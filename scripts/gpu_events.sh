#!/bin/bash
# Event-stream framing CRCs: GPU parity suite, then the framing benchmark on
# the lane-per-buffer scan and (AMDCRC_DEBUG bit 23) on the wave-per-tile list scan.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-events}; mkdir -p $O
ev() { local tag=$1 envs=$2; shift 2; env X=0 $envs timeout -k 10 120 python aws-crt-cpp_amd/tools/bench_eventstream.py "$@" > $O/$tag.json 2> $O/$tag.err && echo "$tag $(cat $O/$tag.json)"; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && tail -1 $O/pytest.log &&
ev small "" &&
ev small_tiles "AMDCRC_DEBUG=8388608" &&
ev tiny "" --messages 524288 --min-bytes 16 --max-bytes 256 &&
ev tiny_tiles "AMDCRC_DEBUG=8388608" --messages 524288 --min-bytes 16 --max-bytes 256 &&
ev medium "" --messages 16384 --min-bytes 1024 --max-bytes 65536 &&
ev small_dev "" --device-frames &&
ev tiny_dev "" --device-frames --messages 524288 --min-bytes 16 --max-bytes 256
