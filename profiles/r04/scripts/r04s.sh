# round 4 (late): staging writes skip the chunks past the item's span in the product -- record-kernel
# tests, A/B against every chunk staged (179 = MODE 39), WAL bench lines
set -o pipefail
O=gpurun_out/r04s; mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 500 $T tests/test_lanespan.py tests/test_log.py tests/test_gpu_parity.py tests/test_sst4k.py > $O/tests_span.log 2>&1 || { echo SPAN_TESTS_FAILED; tail -30 $O/tests_span.log; exit 1; }
tail -1 $O/tests_span.log
timeout -k 10 600 python -u tools/ab_span.py 0,179 wal400,wal1000,wal,wal100,rand300_500,rand64_1000 4 > $O/ab_skiptail_product.log 2>&1 || { echo AB_FAILED; tail $O/ab_skiptail_product.log; exit 1; }
cat $O/ab_skiptail_product.log
