# round 4, third GPU pass: the pre-shifted fold in the product; staging-read addressing variants
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests/test_lanespan.py tests/test_log.py tests/test_gpu_parity.py > $O/tests_span.log 2>&1 || { echo SPAN_TESTS_FAILED; tail -30 $O/tests_span.log; exit 1; }
tail -2 $O/tests_span.log
timeout -k 10 600 python -u tools/ab_span.py 0,162,165,166 wal400,wal1000,wal,wal100,rand300_500,rand64_1000 4 > $O/ab_variants.log 2>&1; echo ab_rc=$?; cat $O/ab_variants.log
timeout -k 10 400 $T tests/test_sst4k.py tests/test_table.py > $O/tests_sst.log 2>&1; echo sst_tests_rc=$?; tail -2 $O/tests_sst.log
timeout -k 10 600 bash tools/profile.sh r04d/prof_verify sst_verify > $O/prof_verify.log 2>&1; echo prof_rc=$?; tail -22 $O/prof_verify.log
