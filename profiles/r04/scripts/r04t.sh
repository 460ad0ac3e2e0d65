# round 4 final: GPU suite, smoke, bench.py as the driver runs it with no flags, the WAL rows
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAILED; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo BENCH_FAILED; tail $O/bench_default.log; exit 1; }
for w in wal wal100 wal400 wal1000; do
  timeout -k 10 300 python bench.py --workload $w --no-copy-inclusive --steps 200 --warmup 100 > $O/bench_$w.log 2>&1 || { echo BENCH_FAILED $w; tail -5 $O/bench_$w.log; exit 1; }
done
grep -h '^{"metric' $O/bench_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['config']['workload'][:14], d['value'], d['roofline']['frac'], d['steps'], d['warmup'])"
