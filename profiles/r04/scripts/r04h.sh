timeout -k 10 900 bash tools/span_pmc.sh r04h 0,169 wal1000,wal100 > gpurun_out/r04h.log 2>&1; rc=$?; tail -3 gpurun_out/r04h.log; exit $rc
