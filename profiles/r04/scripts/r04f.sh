# round 4: LDS / SQ counters of the shipped record kernel on every WAL row
set -o pipefail
timeout -k 10 900 bash tools/counters_span.sh r04f wal400 wal1000 wal wal100 > gpurun_out/r04f_counters.log 2>&1; rc=$?
tail -3 gpurun_out/r04f_counters.log; exit $rc
