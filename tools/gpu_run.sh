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
    cold) step cold 300 python tools/cold_start.py ;;
    cold_variants) step cold_variants 300 python tools/cold_variants.py --variants 0,-1,19,24,13,28,12 ;;
    c2_waves) step ab_c2w 300 python tools/ab_fast.py 0,45,46 8 && step cold_c2w 300 python tools/cold_variants.py --variants 0,45,46,-1 ;;
    counters_c2) step counters_c2 600 bash tools/counters_c2.sh ${TAG}_cntc2 ;;
    cold_q4) step cold_q4 300 python tools/cold_variants.py --variants 0,99,-1 ;;
    ab_c2) step ab_c2 300 python tools/ab_fast.py 0,99 8 ;;
    ab_q4) step ab_q4_sst 300 python tools/ab_sst.py 0,30 && step ab_q4_wal 300 python tools/ab_desc.py 0,42 wal && step ab_q4_desc4k 300 python tools/ab_desc.py 0,43 sst ;;
    ab_q4c3) step ab_q4_c3 300 python tools/ab_desc.py 0,44 c3 ;;
    ab_q4r) step ab_q4r_wal 300 python tools/ab_desc.py 0,42 wal && step ab_q4r_wal_rev 300 python tools/ab_desc.py 42,0 wal && step ab_q4r_desc4k 300 python tools/ab_desc.py 43,0 sst && step ab_q4r_sst 300 python tools/ab_sst.py 30,0 && step ab_q4r_c3 300 python tools/ab_desc.py 44,0 c3 ;;
    lanespan) step lanespan 600 python -u -m pytest tests/test_lanespan.py tests/test_sst4k.py -m gpu -x -v --timeout 200 --timeout-method thread ;;
    ab_lanespan) step ab_lanespan 600 python tools/ab_lanespan.py ;;
    probe_wal100) step probe_wal100 900 bash tools/counters_probe.sh ${TAG}_probe100 wal100 0 64 67 ;;
    probe_wal400) step probe_wal400 900 bash tools/counters_probe.sh ${TAG}_probe400 wal400 0 64 67 ;;
    counters_span) step counters_span 900 bash tools/counters_span.sh ${TAG}_span wal100 wal400 ;;
    integ) step integ 600 python -u -m pytest tests/test_integration.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    fullsize) step fullsize 600 python -u -m pytest tests/test_full_size.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "full_size or host_" ;;
    bench_driver) step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --diag ;;
    prof_wal) step prof_wal100 500 bash tools/profile.sh ${TAG}_prof_wal100 wal100 && step prof_wal400 500 bash tools/profile.sh ${TAG}_prof_wal400 wal400 && step prof_wal1000 500 bash tools/profile.sh ${TAG}_prof_wal1000 wal1000 ;;
    bench_wal) step bench_wal100 300 python bench.py --workload wal100 --no-copy-inclusive && step bench_wal400 300 python bench.py --workload wal400 --no-copy-inclusive && step bench_wal1000 300 python bench.py --workload wal1000 --no-copy-inclusive ;;
    copyinc) step copyinc 600 python tools/copy_inclusive.py ;;
    prof_c2) step prof_c2 700 bash tools/profile.sh ${TAG}_prof_c2 c2 ;;
    prof_rows) step prof_c3 700 bash tools/profile.sh ${TAG}_prof_c3 c3 && step prof_sst_verify 700 bash tools/profile.sh ${TAG}_prof_sst_verify sst_verify && step prof_sstable 700 bash tools/profile.sh ${TAG}_prof_sstable sstable && step prof_wal 700 bash tools/profile.sh ${TAG}_prof_wal wal ;;
    prof_list) for w in ${PROF_WL:-c2}; do step prof_$w 700 bash tools/profile.sh ${TAG}_prof_$w $w || exit 1; done ;;
    ab_seal) step ab_seal 600 python tools/ab_sst.py 0,37,39 ;;
    ab_waves2) step ab_waves2 600 python tools/ab_waves.py ;;
    ab_hints) step ab_hints 600 python tools/ab_hints.py ;;
    ab_waves) step ab_waves 600 python tools/ab_sst.py 0,127,128 && step ab_waves_rev 600 python tools/ab_sst.py 128,127,0 ;;
    vtool) step vtool 900 bash tools/verify_tool_bench.sh ${TAG}_vtool 1000000 ;;
    vtool10m) step vtool10m 1000 bash tools/verify_tool_bench.sh ${TAG}_vtool10m 10000000 ;;
    seal_price) step seal_price 600 python tools/seal_price.py ;;
    lanespan_var) step lanespan_var 600 python -u -m pytest tests/test_lanespan.py -m gpu -x -q --timeout 200 --timeout-method thread ;;
    ab_var) step ab_var 900 python tools/ab_span.py 0,125 rand300_500,rand64_1000,rand32_256,rand1_512,rand1000_1152,wal100,wal400,wal1000,wal 4 ;;
    seal_cal) step seal_cal 600 python tools/seal_price.py 0,140,141,142,33 ;;
    seal_cal2) step seal_cal2 600 python tools/seal_price.py 0,140,141,143,144,145,146,147 ;;
    seal_cal3) step seal_cal3 600 python tools/seal_price.py 0,140,141,148,149,150,151 ;;
    ab_seal_price) step ab_seal_price 600 python tools/ab_sst.py 0,94,95,96 && step ab_seal_price_rev 600 python tools/ab_sst.py 96,95,94,0 ;;
    ab_seal_orders) step ab_so1 600 python tools/ab_sst.py 0,94,95 && step ab_so2 600 python tools/ab_sst.py 95,94,0 && step ab_so3 600 python tools/ab_sst.py 94,0 ;;
    bench_rows) for w in sst_verify sst_seal sst_crc wal sstable c3; do step bench_$w 300 python bench.py --workload $w --no-copy-inclusive --steps 50 || exit 1; done ;;
    bench_rows4) for w in c3 sstable sst_verify sst_seal sst_crc wal wal100 wal400 wal1000; do step bench_$w 300 python bench.py --workload $w --no-copy-inclusive --steps 50 || exit 1; done ;;
    bench_driver3) for i in 1 2 3; do step bench_driver_$i 300 python bench.py || exit 1; done ;;
    bench_sst3) for w in sst_verify sst_crc sstable; do step bench3_$w 300 python bench.py --workload $w --no-copy-inclusive --steps 50 || exit 1; done ;;
    bench_sst) step bench_sst 600 python bench.py --workload sstable --no-cpu-baseline --no-copy-inclusive ;;
    bench_c3) step bench_c3 600 python bench.py --workload c3 --no-copy-inclusive --steps 10 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
