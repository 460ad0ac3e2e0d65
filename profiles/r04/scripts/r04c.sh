# round 4, second GPU pass: record-kernel variants on the dword-read base; two-launch seal counters
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 600 python -u tools/ab_span.py 0,162,163,164 wal400,wal1000,wal,wal100,rand300_500,rand64_1000 4 > $O/ab_variants.log 2>&1; echo ab_rc=$?; cat $O/ab_variants.log
timeout -k 10 600 bash tools/profile.sh r04c/prof_seal2 sst_seal2 > $O/prof_seal2.log 2>&1; echo prof_rc=$?; tail -25 $O/prof_seal2.log
