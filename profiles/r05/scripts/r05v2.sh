# round 5: the record kernel's parts on every WAL row (63 loads + staging, 64 hash alone, 67 bookkeeping alone)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_span.py 0,63,64,67 wal100,wal400,wal1000,wal 6 > gpurun_out/r05v2_parts.log 2>&1
