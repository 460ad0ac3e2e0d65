# round 4: record kernel -- p-word selects on every step, branch-free: wave masks (174 = MODE 34),
# plain selects (175 = MODE 35); 115 = no selects at all (pricing, wrong CRCs)
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 900 python -u tools/ab_span.py 0,174,175,115 wal400,wal1000,wal,wal100,rand300_500,rand64_1000 4 > $O/ab_nog.log 2>&1; rc=$?; echo ab_rc=$rc; cat $O/ab_nog.log; exit $rc
