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
P="--steps 20 --warmup 20 --only-coalesced --branches 1 --no-configs --no-c4 --no-cpu-baseline --e2e-batches 0 --timing-launches 16"
rc=0
for s in "$@"; do
  case $s in
    test)  step 900 $O/pytest.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider; rc=$?; tail -3 $O/pytest.log ;;
    tsel)  step 600 $O/pytest_sel.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "${TESTK:-xcd}"; rc=$?; tail -3 $O/pytest_sel.log ;;
    smoke) step 180 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; tail -2 $O/smoke.log ;;
    bench) step 400 $O/bench.log python -u bench.py ${BENCH_ARGS:-}; rc=$?; tail -1 $O/bench.log ;;
    driver*) t0=$(date +%s); step 400 $O/$s.log python -u bench.py --gpus 1 --steps 20 --warmup 5; rc=$?; echo "[driver] wall $(( $(date +%s) - t0 )) s" >> $O/$s.log; grep '^{' $O/$s.log | cut -c1-400; tail -1 $O/$s.log ;;
    # the N > 1 rank path rehearsed on the one GPU: two gloo ranks, the full bench (C4 legs, CPU baseline)
    gloo2) t0=$(date +%s); step 600 $O/gloo2.log python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --e2e-batches 0; rc=$?; echo "[gloo2] wall $(( $(date +%s) - t0 )) s" >> $O/gloo2.log; grep '^{' $O/gloo2.log | cut -c1-300; tail -1 $O/gloo2.log ;;
    # the timed region decomposed: kernel + HIP API trace of the driver's timed region (legs trimmed)
    trace) (cd /tmp && step 300 $O/trace.log rocprofv3 --kernel-trace --hip-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-configs --no-cpu-baseline --e2e-batches 0); rc=$? ;;
    # kernel trace of the driver's exact command
    kprof) (cd /tmp && step 420 $O/kprof.log rocprofv3 --kernel-trace --stats -d $O/kprof -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5); rc=$? ;;
    prof)  (cd /tmp && step 300 $O/prof.log rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py $P ${PROF_ARGS:-}); rc=$? ;;
    pmc)   (cd /tmp && step 120 $O/pmc_fetch.log timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py $P ${PROF_ARGS:-}); rc=$? ;;
    # the driver-shaped region per submission path, under HIP runtime settings (one process each)
    probe) for v in ${PROBE_ENVS:-""}; do
             step 120 $O/probe.log.tmp env $v python -u aws-crt-cpp_amd/tools/overhead_probe.py 20 40; rc=$?; cat $O/probe.log.tmp >> $O/probe.log
             [ $rc -ne 0 ] && break; done; grep '^{' $O/probe.log | cut -c1-600 ;;
    # kernel traces of the event-stream bench and of the ragged-list probe
    esprof) (cd /tmp && step 180 $O/esprof.log rocprofv3 --kernel-trace --stats -d $O/esprof -o run --output-format csv -- python3 $R/aws-crt-cpp_amd/tools/bench_eventstream.py --device-frames); rc=$? ;;
    listprof) (cd /tmp && step 180 $O/listprof.log rocprofv3 --kernel-trace --stats -d $O/listprof -o run --output-format csv -- python3 $R/aws-crt-cpp_amd/tools/list_probe.py ${LIST_ALG:-crc32c}); rc=$? ;;
    sq)    step 300 $O/sq.log env TAG=${TAG}/sq bash scripts/pmc_sq.sh; rc=$?; tail -1 $O/sq.log ;;
    es)    step 180 $O/es.log python -u aws-crt-cpp_amd/tools/bench_eventstream.py --device-frames; rc=$?; grep '^{' $O/es.log | cut -c1-500 ;;
    # SQ issue / stall / LDS counters of the event-stream framing kernel (one pass)
    sqes)  (cd /tmp && step 120 $O/sqes.log timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/sqes -o run --output-format csv -- python3 $R/aws-crt-cpp_amd/tools/bench_eventstream.py --device-frames --steps 12 --timing-launches 4); rc=$? ;;
    sqes2) (cd /tmp && step 120 $O/sqes2.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES TCP_TCC_READ_REQ_sum TA_BUSY_avr GRBM_GUI_ACTIVE -d $O/sqes2 -o run --output-format csv -- python3 $R/aws-crt-cpp_amd/tools/bench_eventstream.py --device-frames --steps 12 --timing-launches 4); rc=$? ;;
    ablist) step 900 $O/ablist.log env TAG=${TAG}/ablist VARIANTS="${VARIANTS:-A B C D}" REPS=${REPS:-2} bash scripts/ab_listprobe.sh; rc=$?; cat $O/ablist.log ;;
    readpat) step 150 $O/readpat.log bash -c "experiments/build/readpattern 1280 16 && experiments/build/readpattern 512 16"; rc=$?; cat $O/readpat.log ;;
    # A/B of library builds on the driver-shaped bench (ab/lib$v.so for v in $VARIANTS)
    abx)   step 900 $O/abx.log env TAG=${TAG}/abx VARIANTS="${XVARIANTS:-R X}" REPS=${REPS:-3} bash scripts/ab_lib.sh python -u bench.py --steps 20 --warmup 5 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 8; rc=$?; cat $O/abx.log ;;
    # the same on the C5 CRC64NVME launch (8 x 64 MiB)
    ab64)  step 900 $O/ab64.log env TAG=${TAG}/ab64 VARIANTS="${X64VARIANTS:-R W}" REPS=${REPS:-3} bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --steps 20 --warmup 5 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 8; rc=$?; cat $O/ab64.log ;;
    ab64c1) step 900 $O/ab64c1.log env TAG=${TAG}/ab64c1 VARIANTS="${X64VARIANTS:-R W}" REPS=${REPS:-3} bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --steps 20 --warmup 5 --coalesce 1 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 8; rc=$?; cat $O/ab64c1.log ;;
    # the GPU parity tests that cover the uniform-batch scans, on variant $XLIB (then the release build back)
    xtests) cp aws-crt-cpp_amd/lib/libaws-checksums-amd.so /tmp/librel.so && cp ab/lib${XLIB:-X}.so aws-crt-cpp_amd/lib/libaws-checksums-amd.so &&
            step 600 $O/xtests.log python -u -m pytest tests/test_gpu_parity.py tests/test_queue.py tests/test_multipart.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider; rc=$?;
            cp /tmp/librel.so aws-crt-cpp_amd/lib/libaws-checksums-amd.so; tail -3 $O/xtests.log ;;
    # event-stream bench on library variants (ab/lib$v.so, v in $ESVARIANTS), then the release build back
    abes)  cp aws-crt-cpp_amd/lib/libaws-checksums-amd.so /tmp/librel.so; rc=0
           for v in ${ESVARIANTS:-R B}; do for r in 1 2; do cp ab/lib$v.so aws-crt-cpp_amd/lib/libaws-checksums-amd.so &&
             step 180 $O/abes_${v}_$r.log python -u aws-crt-cpp_amd/tools/bench_eventstream.py --device-frames || { rc=$?; break 2; }
             echo "$v $r $(grep '^{' $O/abes_${v}_$r.log | cut -c180-420)"; done; done
           cp /tmp/librel.so aws-crt-cpp_amd/lib/libaws-checksums-amd.so ;;
    ingest) step 300 $O/ingest.log env AWS_CRT_AMD_INGEST_TRACE=${INGEST_TRACE:-0} python -u aws-crt-cpp_amd/tools/ingest_probe.py; rc=$?; grep '^{' $O/ingest.log | tail -1 | cut -c1-300 ;;
    tests:*) step 900 $O/pytest_sel.log python -u -m pytest $(echo ${s#tests:} | tr , " ") -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider; rc=$?; tail -3 $O/pytest_sel.log ;;
    py:*)  n=$(basename ${s#py:} .py); step 600 $O/$n.log python -u ${s#py:}; rc=$?; tail -5 $O/$n.log ;;
    # the value-only ABI's small-call latency (C++), pointer cache on and off
    lat)   step 120 $O/lat.log bash -c "experiments/build/abi_latency 200000 && AWS_CRT_AMD_PTR_CACHE=0 experiments/build/abi_latency 200000"; rc=$?; cat $O/lat.log ;;
    # the multi-GPU rank path rehearsed on the box's one GPU (two gloo ranks) and the in-process fan-out
    ranks) step 300 $O/ranks.log bash -c "python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-configs --e2e-batches 0 --no-cpu-baseline && python -u bench.py --inproc --gpus 1 --steps 20 --warmup 5"; rc=$?; grep '^{' $O/ranks.log | cut -c1-600 ;;
    # every config leg's kernel fraction (no CPU baseline, no host legs)
    legs)  step 400 $O/legs.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-batches 0; rc=$?; grep '^{' $O/legs.log | cut -c1-300 ;;
    # FETCH_SIZE of the C5 CRC64NVME launch (8 x 64 MiB, one batch per launch)
    legsx) step 400 $O/legsx.log env AWS_CRT_AMD_X64_TRACE=1 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-batches 0; rc=$?; grep '^\[x64\]' $O/legsx.log | tail -4 ;;
    stamps) step 180 $O/stamps.log python -u aws-crt-cpp_amd/tools/stamp_probe.py ${STAMP_REPS:-5}; rc=$?; grep -c '^{' $O/stamps.log ;;
    # effective shader clock per dispatch (GRBM_GUI_ACTIVE / duration): CRC64 C5 20-batch vs single, C2
    clk64) (cd /tmp && step 120 $O/clk64.log timeout -s KILL 100 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d $O/clk64 -o run --output-format csv -- python3 $R/bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --steps 20 --warmup 2 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 4); rc=$? ;;
    clk32) (cd /tmp && step 120 $O/clk32.log timeout -s KILL 100 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d $O/clk32 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 4); rc=$? ;;
    lists) step 240 $O/lists.log bash -c "python -u aws-crt-cpp_amd/tools/list_probe.py crc32c && python -u aws-crt-cpp_amd/tools/list_probe.py crc64nvme"; rc=$?; grep '^{' $O/lists.log | cut -c1-300 ;;
    pmc5)  (cd /tmp && step 120 $O/pmc5_fetch.log timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $O/pmc5_fetch -o run --output-format csv -- python3 $R/bench.py --alg crc64nvme --buffers 8 --buffer-bytes 67108864 --batches 2 --coalesce 1 --steps 12 --warmup 2 --only-coalesced --branches 1 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 4); rc=$? ;;
    # A/B of library builds on the C4 shard CRC64NVME launch (131072 x 8 KiB, crc64_rows16_kernel)
    abr16) step 900 $O/abr16.log env TAG=${TAG}/abr16 VARIANTS="${R16VARIANTS:-R OLD}" REPS=${REPS:-3} bash scripts/ab_lib.sh python -u bench.py --alg crc64nvme --buffers 131072 --buffer-bytes 8192 --batches 2 --coalesce 1 --steps 20 --warmup 5 --no-configs --no-cpu-baseline --e2e-batches 0 --timing-launches 8; rc=$?; cat $O/abr16.log ;;
    # CRC64NVME vs CRC32C vs the read ceiling, same launch shapes (round 6), and its counter passes
    c64)   step 300 $O/c64.log python -u aws-crt-cpp_amd/tools/crc64_probe.py ${C64_ARGS:-}; rc=$?; grep '^{' $O/c64.log | cut -c1-400 ;;
    pmc64) step 420 $O/pmc64.log env TAG=${TAG}/pmc64 bash scripts/pmc_crc64.sh; rc=$?; tail -2 $O/pmc64.log ;;
    # the LDS chain microbenchmark of the CRC64 row step (experiments/crc64_rowbench.hip)
    rowb)  step 120 $O/rowb.log experiments/build/crc64_rowbench; rc=$?; cat $O/rowb.log ;;
    # A/B of checksum-library builds (ab/lib$v.so) on any command: ABVARIANTS, ABCMD
    abc)   step 900 $O/abc.log env TAG=${TAG}/abc VARIANTS="${ABVARIANTS:-R X}" REPS=${REPS:-2} bash scripts/ab_cmd.sh $ABCMD; rc=$?; cat $O/abc.log ;;
    pmces) step 600 $O/pmces.log env TAG=${TAG}/pmces VARIANTS="${ESVARIANTS:-C ESL}" bash scripts/pmc_es.sh; rc=$?; tail -2 $O/pmces.log ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  [ $rc -ne 0 ] && { echo "session stopped at $s rc=$rc"; exit $rc; }
done
echo "session ok"
