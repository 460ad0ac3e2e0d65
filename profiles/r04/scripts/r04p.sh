# round 4 (late): the branch-free p-word selects in the product -- record-kernel tests, A/B against the
# G-bounded form (176 = MODE 36), WAL bench lines
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 500 $T tests/test_lanespan.py tests/test_log.py tests/test_gpu_parity.py > $O/tests_span.log 2>&1 || { echo SPAN_TESTS_FAILED; tail -30 $O/tests_span.log; exit 1; }
tail -2 $O/tests_span.log
timeout -k 10 600 python -u tools/ab_span.py 0,176 wal400,wal1000,wal,wal100,rand300_500,rand64_1000 4 > $O/ab_nog_product.log 2>&1 || { echo AB_FAILED; tail $O/ab_nog_product.log; exit 1; }
cat $O/ab_nog_product.log
for w in wal wal100 wal400 wal1000; do
  timeout -k 10 300 python bench.py --workload $w --no-copy-inclusive --steps 50 > $O/bench_$w.log 2>&1 || { echo BENCH_FAILED $w; tail -5 $O/bench_$w.log; exit 1; }
done
grep -h '^{"metric' $O/bench_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['config']['workload'][:12], d['value'], d['roofline']['frac'])"
