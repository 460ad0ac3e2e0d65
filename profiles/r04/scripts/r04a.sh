set -o pipefail
mkdir -p gpurun_out/r04a
timeout -k 10 300 python -u -m pytest tests/test_lanespan.py tests/test_log.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r04a/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r04a/tests.log; exit 1; }
tail -3 gpurun_out/r04a/tests.log
timeout -k 10 400 python -u tools/ab_span.py 0,160 wal400,wal1000,wal,wal100 4 > gpurun_out/r04a/ab_pairs.log 2>&1
cat gpurun_out/r04a/ab_pairs.log
timeout -k 10 300 python -u -m pytest tests/test_integration.py -x -q --timeout 200 --timeout-method thread -m gpu -k "leveldb_verify_batched" > gpurun_out/r04a/tests_verify.log 2>&1; echo verify_rc=$?; tail -3 gpurun_out/r04a/tests_verify.log
timeout -k 10 300 python -u -m pytest tests/test_shard.py -x -q --timeout 200 --timeout-method thread -m gpu -k "rccl" > gpurun_out/r04a/tests_rccl.log 2>&1; echo rccl_rc=$?; tail -3 gpurun_out/r04a/tests_rccl.log
timeout -k 10 300 python -u -m pytest tests/test_scalar_server.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r04a/tests_server.log 2>&1; echo server_rc=$?; tail -5 gpurun_out/r04a/tests_server.log
