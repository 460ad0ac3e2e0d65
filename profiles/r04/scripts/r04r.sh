# round 4 (late): record kernel -- chunks past the item's span neither loaded nor staged (177 = MODE 37)
# or only not staged (178 = MODE 38); exactness test of every round-4 form first
set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_lanespan.py -k round4 > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python -u tools/ab_span.py 0,177,178 wal400,wal1000,wal,wal100,rand300_500,rand64_1000 4 > $O/ab_skiptail.log 2>&1; rc=$?; echo ab_rc=$rc; cat $O/ab_skiptail.log; exit $rc
