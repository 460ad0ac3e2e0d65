# round 5: long blocks on the DMA route too -- host-path GPU tests (incl. the small-group child runs),
# then the long-block cost on both routes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_table.py tests/test_sst4k.py tests/test_integration.py tests/test_capi.py \
  tests/test_gpu_parity.py tests/test_sst_files.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05ue_tests.log 2>&1 \
  || { tail -40 gpurun_out/r05ue_tests.log; exit 1; }
tail -2 gpurun_out/r05ue_tests.log
timeout -k 10 300 python tools/long_block_cost.py > gpurun_out/r05ue_long_block_cost.log 2>&1
