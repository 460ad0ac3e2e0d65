# round 5: price the record kernel's fold operators (127: free, 128: 8 conflict-free lookups each)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_span.py 0,127,128 wal400,wal1000,wal100,wal 6 > gpurun_out/r05r_fold_price.log 2>&1
