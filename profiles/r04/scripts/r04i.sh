# round 4: where the record kernel's VALU and LDS cycles go -- the shipped kernel (0) against its loads +
# staging alone (63), its hash alone over stale staging (64) and its bookkeeping alone (67)
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 600 python -u tools/ab_span.py 0,169,63,64,67 wal1000,wal400,wal100,wal 3 > $O/ab_parts.log 2>&1 || { echo AB_FAILED; tail $O/ab_parts.log; exit 1; }
cat $O/ab_parts.log
timeout -k 10 900 bash tools/span_pmc.sh r04i_pmc 0,63,64,67 wal1000,wal400 > $O/pmc.log 2>&1; rc=$?; tail -1 $O/pmc.log; exit $rc
