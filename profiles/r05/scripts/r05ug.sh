# round 5: the cross-lane pre-shift's lookups EXEC-masked to the lanes that use them (133) vs shipped, both orders
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_span.py 0,133 wal400,wal1000,wal,rand300_500,wal100 8 > gpurun_out/r05ug_ab_slotmask.log 2>&1 && \
timeout -k 10 400 python tools/ab_span.py 133,0 wal400,wal1000,wal,rand300_500,wal100 8 >> gpurun_out/r05ug_ab_slotmask.log 2>&1
