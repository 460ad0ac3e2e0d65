# round 5: 11 waves x 8928-B regions for the <= 256-B and 1024..1152-B classes -- parity, then A/B
# against 10 x 9 KiB (w10 = the previous commit's library), both orders
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_lanespan.py tests/test_log.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05aa_tests.log 2>&1 || { tail -30 gpurun_out/r05aa_tests.log; exit 1; }
tail -2 gpurun_out/r05aa_tests.log
AB_VARIANTS=0,w10/0 AB_WL=wal100,wal,rand32_256,rand1000_1152 AB_ROUNDS=6 bash tools/gpu_run.sh r05aa ab_vs || exit 1
AB_VARIANTS=w10/0,0 AB_WL=wal100,wal AB_ROUNDS=6 bash tools/gpu_run.sh r05ab ab_vs
