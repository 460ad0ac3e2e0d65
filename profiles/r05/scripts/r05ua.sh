# round 5: long blocks out of the zero-copy sst kernel (span launches) -- the host-path GPU tests, then
# the engine's 10 M fill with PDB_SEAL_STAMPS
set -o pipefail
O=gpurun_out/r05ua; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_table.py tests/test_sst4k.py tests/test_integration.py tests/test_capi.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
DB=/tmp/pdb_r05ua_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
PDB_SEAL_STAMPS=$O/engine_stamps.csv timeout -k 10 300 integration/_build/pdb_dbbench_gpu_table --benchmarks=fillrandom \
  --num=10000000 --value_size=1024 --db=$DB/x > $O/fill.log 2>&1
