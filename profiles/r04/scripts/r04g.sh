# round 4: record kernel -- lock-step staging reads rotated over chain slots by bank class (MODE 29)
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 900 python -u tools/ab_span.py 0,169 wal100,wal1000,wal,rand32_256,rand64_1000,rand1000_1152,wal700 4 > $O/ab_rot.log 2>&1; rc=$?; echo ab_rc=$rc; cat $O/ab_rot.log; exit $rc
