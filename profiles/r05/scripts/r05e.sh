# round 5: interleaved queues (16, batch kQ j + x) -- lanespan tests, then A/B vs the workgroup-local
# distribution, the pattern A/B, clocks
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_lanespan.py tests/test_log.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python tools/ab_span.py 0,183,184,185 wal100,wal400,wal1000,wal 4 > $O/ab_queues.log 2>&1 || exit 1
timeout -k 10 300 python tools/span_clock.py wal1000,wal100 3 > $O/span_clock.log 2>&1 || exit 1
