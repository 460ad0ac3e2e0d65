# round 5: shader clock of the record kernel vs its parts (tools/span_clock.py)
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 300 python tools/span_clock.py wal1000,wal100 3 > $O/span_clock.log 2>&1 || exit 1
