#!/usr/bin/env bash
# tools/rows_bench.sh -- on the GPU box: GPU tests, then bench.py over the SURVEY §8(f) row workloads
# (sst_verify, sst_seal, wal) and the sstable / c3 layouts; logs under gpurun_out/rows_*.log.
set -u
mkdir -p gpurun_out
timeout -k 10 250 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rows_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rows_tests.log; [ $rc -ne 0 ] && exit $rc
for w in sst_verify sst_seal wal sstable c3; do
  timeout -k 10 300 python bench.py --workload $w --no-copy-inclusive --steps 50 > gpurun_out/rows_$w.log 2>&1; rc=$?
  tail -1 gpurun_out/rows_$w.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
done
exit 0
