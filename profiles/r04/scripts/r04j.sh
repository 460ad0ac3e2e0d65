# round 4: record kernel -- one item's loads in flight (MODE 30, half the staging registers) and, with
# the registers that frees, 13 waves x 7-KiB regions (MODE 31)
set -o pipefail
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 900 python -u tools/ab_span.py 0,170,171 wal400,wal1000,wal,wal100,rand300_500,rand64_1000 4 > $O/ab_onedeep.log 2>&1; rc=$?; echo ab_rc=$rc; cat $O/ab_onedeep.log; exit $rc
