# round 4: opaque-base staging reads in the product; one-compare p-word selects (A/B)
set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests/test_lanespan.py tests/test_log.py tests/test_gpu_parity.py > $O/tests_span.log 2>&1 || { echo SPAN_TESTS_FAILED; tail -30 $O/tests_span.log; exit 1; }
tail -2 $O/tests_span.log
timeout -k 10 600 python -u tools/ab_span.py 0,167,168 wal400,wal1000,wal,wal100,rand300_500,rand64_1000 4 > $O/ab_variants.log 2>&1; echo ab_rc=$?; cat $O/ab_variants.log
