# round 4, first GPU pass: parity of every changed path, then the record-kernel A/B and the rows
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests/test_lanespan.py tests/test_log.py > $O/tests_span.log 2>&1 || { echo SPAN_TESTS_FAILED; tail -30 $O/tests_span.log; exit 1; }
tail -2 $O/tests_span.log
timeout -k 10 400 $T tests/test_sst4k.py -k "seal" > $O/tests_seal.log 2>&1 || { echo SEAL_TESTS_FAILED; tail -30 $O/tests_seal.log; exit 1; }
tail -2 $O/tests_seal.log
timeout -k 10 300 $T tests/test_scalar_server.py > $O/tests_server.log 2>&1; echo server_rc=$?; tail -3 $O/tests_server.log
timeout -k 10 300 $T tests/test_integration.py -k "leveldb_verify_batched" > $O/tests_verify.log 2>&1; echo verify_rc=$?; tail -3 $O/tests_verify.log
timeout -k 10 300 $T tests/test_shard.py -k "rccl" > $O/tests_rccl.log 2>&1; echo rccl_rc=$?; tail -3 $O/tests_rccl.log
timeout -k 10 500 python -u tools/ab_span.py 0,160,162,163 wal400,wal1000,wal,wal100,rand300_500,rand64_1000 4 > $O/ab_pairs.log 2>&1; echo ab_rc=$?; cat $O/ab_pairs.log
for w in sst_seal sst_seal2 c3 sstable; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 50 --warmup 20 --no-cpu-baseline --no-copy-inclusive > $O/bench_$w.log 2>&1; echo "bench $w rc=$?"
  python - $O/bench_$w.log <<'PY'
import json,sys
for ln in open(sys.argv[1]):
    if ln.startswith('{"metric"'):
        d=json.loads(ln); print(d["config"]["workload"][:40], d["roofline"]["frac"], (d.get("steady_state") or {}).get("frac"), json.dumps(d.get("pattern_ceiling")))
PY
done
timeout -k 10 240 python -u tools/scalar_phases.py $O/scalar_phases.json 20000 > $O/scalar_phases.log 2>&1; echo phases_rc=$?; tail -40 $O/scalar_phases.log
