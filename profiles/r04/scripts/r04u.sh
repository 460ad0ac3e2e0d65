# round 4 final: LDS / SQ counters of the final shipped record kernel on every WAL row
set -o pipefail
timeout -k 10 900 bash tools/counters_span.sh r04u wal400 wal1000 wal wal100 > gpurun_out/r04u_counters.log 2>&1; rc=$?
tail -3 gpurun_out/r04u_counters.log; exit $rc
