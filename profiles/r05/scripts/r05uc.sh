# round 5: long blocks in two launches per batch (one descriptor launch over all their 4-KiB pieces,
# one combine) -- host-path GPU tests, then a stamped 10 M fill and the split / none A/B
set -o pipefail
O=gpurun_out/r05uc; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_table.py tests/test_sst4k.py tests/test_integration.py tests/test_capi.py -m gpu -x -v \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
DB=/tmp/pdb_r05uc_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
fill() {  # name env...
  local name=$1; shift
  rm -rf $DB/x
  env "$@" timeout -k 10 300 integration/_build/pdb_dbbench_gpu_table --benchmarks=fillrandom --num=10000000 \
    --value_size=1024 --db=$DB/x > $O/$name.log 2>&1 || return 1
  grep -a "micros/op" $O/$name.log | head -1
}
fill many_a PDB_SEAL_STAMPS=$O/many_a_stamps.csv && fill none_a PDB_LONG_BLOCK=0 && fill many_b PDB_X=1
