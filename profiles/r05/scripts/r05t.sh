# round 5: price the record kernel's staging stores (131) and its fold (127)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_span.py 0,131,127 wal400,wal1000,wal,wal100 6 > gpurun_out/r05t_store_price.log 2>&1
