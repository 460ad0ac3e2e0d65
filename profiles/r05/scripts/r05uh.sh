# round 5: the record kernel's exact diagnostics variants (125, 133) against the oracle
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_lanespan.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r05uh_lanespan.log 2>&1
