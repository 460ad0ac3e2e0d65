# round 5: price the record kernel's fold (127 free, 129 no dependence between lookups, 130 cross-lane free)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_span.py 0,127,129,130 wal400,wal1000,wal 6 > gpurun_out/r05s_fold_price2.log 2>&1
