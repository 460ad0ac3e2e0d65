# round 5: the cost of one long block in a 16-MiB host seal / verify batch, both routes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/long_block_cost.py > gpurun_out/r05ud_long_block_cost.log 2>&1
