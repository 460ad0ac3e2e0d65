#!/usr/bin/env bash
# tools/gpu_run.sh -- run on the GPU box via gpurun: GPU tests, then a bench line.
# Each GPU step has its own time limit; a fault / abort / timeout (rc >= 124 or signal)
# stops the script before any further GPU work.  A plain test failure (rc 1) does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG="${1:-run}"
shift || true
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/${TAG}_steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/${TAG}_steps.log
  tail -5 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case "$s" in
    tests) step tests 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench_driver) step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench) step bench 600 python bench.py --diag ;;
    cold) step cold 300 python tools/cold_start.py ;;
    lanespan) step lanespan 600 python -u -m pytest tests/test_lanespan.py tests/test_log.py -m gpu -x -v --timeout 200 --timeout-method thread ;;
    integ) step integ 600 python -u -m pytest tests/test_integration.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    fullsize) step fullsize 600 python -u -m pytest tests/test_full_size.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "full_size or host_" ;;
    # the record kernel: 50-step bench lines, parts / distribution A/B, clocks, counters
    bench_wal) for w in wal100 wal400 wal1000 wal; do step bench_$w 300 python bench.py --workload $w --no-copy-inclusive --steps 50 || exit 1; done ;;
    ab_span) step ab_span 600 python tools/ab_span.py 0,63,64,67 wal100,wal400,wal1000,wal 6 ;;
    ab_vs) step ab_vs 900 python tools/ab_span.py ${AB_VARIANTS:-0,wgl/0} ${AB_WL:-wal100,wal400,wal1000,wal,rand300_500,rand64_1000} ${AB_ROUNDS:-6} ;;
    span_clock) step span_clock 600 python tools/span_clock.py wal100,wal400,wal1000,wal 3 ;;
    counters_span) step counters_span 900 bash tools/counters_span.sh ${TAG}_span wal100 wal400 wal1000 wal ;;
    prof_wal) for w in wal100 wal400 wal1000 wal; do step prof_$w 500 bash tools/profile.sh ${TAG}_prof_$w $w || exit 1; done ;;
    # every §8(f) row and C3, 50-step bench lines and rocprof evidence
    bench_rows) for w in c3 sstable sst_verify sst_seal sst_crc sst_tables wal wal100 wal400 wal1000; do step bench_$w 300 python bench.py --workload $w --no-copy-inclusive --steps 50 || exit 1; done ;;
    prof_c2) step prof_c2 700 bash tools/profile.sh ${TAG}_prof_c2 c2 ;;
    prof_list) for w in ${PROF_WL:-c2}; do step prof_$w 700 bash tools/profile.sh ${TAG}_prof_$w $w || exit 1; done ;;
    copyinc) step copyinc 600 python tools/copy_inclusive.py ;;
    sealb) step sealb 300 python tools/seal_batches.py ${SEAL_MIB:-4,16,32} ;;
    ab_sst) step ab_sst 600 python tools/ab_sst.py 0,72 ;;
    # the engine (BASELINE configs 1 / 5, §8(f) row 1)
    vtool) step vtool 900 bash tools/verify_tool_bench.sh ${TAG}_vtool 1000000 ;;
    vtool10m) step vtool10m 1000 bash tools/verify_tool_bench.sh ${TAG}_vtool10m 10000000 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
