# round 4: pricing on the shipped kernel (wrong CRCs by design): conflict-free staging reads (113),
# + conflict-free fold-operator lookups (114), no p-word selects (115)
set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 900 python -u tools/ab_span.py 0,113,114,115 wal400,wal1000,wal,wal100 4 > $O/ab_pricing.log 2>&1; rc=$?; echo ab_rc=$rc; cat $O/ab_pricing.log; exit $rc
