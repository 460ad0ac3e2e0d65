# round 5: price the chains' staging reads as 16-B LDS reads (132), against the shipped kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_span.py 0,132 wal400,wal1000,wal,wal100 6 > gpurun_out/r05w2_read128_price.log 2>&1
