# round 4: record kernel -- p-word selects as wave masks (inverse ballot; MODE 32)
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 900 python -u tools/ab_span.py 0,172 wal400,wal1000,wal,wal100,rand300_500,rand64_1000 4 > $O/ab_masksel.log 2>&1; rc=$?; echo ab_rc=$rc; cat $O/ab_masksel.log; exit $rc
