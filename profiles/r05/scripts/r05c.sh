# round 5: record kernel on device-wide work queues + pruned diagnostics -- full GPU suite, then
# A/B of the queues vs the round-4 distribution, clocks, 50-step bench lines
set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python tools/ab_span.py 0,183 wal100,wal400,wal1000,wal 6 > $O/ab_queues.log 2>&1 || exit 1
timeout -k 10 300 python tools/span_clock.py wal1000,wal100 3 > $O/span_clock.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_pattern.py 21,23 6 > $O/ab_pattern.log 2>&1 || exit 1
for w in wal100 wal400 wal1000 wal; do
  timeout -k 10 200 python bench.py --workload $w --no-copy-inclusive --no-cpu-baseline --steps 50 > $O/bench_$w.log 2>&1 || exit 1
done
