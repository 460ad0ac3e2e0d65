# round 5: tail work stealing in the record kernel -- parity (record kernel, concurrent streams, graph
# capture), then A/B against no stealing (183), both orders, and the per-wave end distribution
set -o pipefail
O=gpurun_out; 
timeout -k 10 600 python -u -m pytest tests/test_lanespan.py tests/test_log.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r05z_tests.log 2>&1 || { tail -30 $O/r05z_tests.log; exit 1; }
tail -2 $O/r05z_tests.log
AB_VARIANTS=0,183 AB_WL=wal100,wal400,wal1000,wal,rand300_500,rand64_1000 AB_ROUNDS=6 bash tools/gpu_run.sh r05z ab_vs || exit 1
bash tools/gpu_run.sh r05z span_clock
