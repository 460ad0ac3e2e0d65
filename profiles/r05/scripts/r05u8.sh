# round 5: zero-copy seals after 0..500 ms of idle GPU (tools/seal_gaps.py), and the engine's 10 M fill
# with PDB_SEAL_STAMPS (phases + page-locking allocations so far)
set -o pipefail
O=gpurun_out/r05u8; mkdir -p $O
PDB_SEAL_STAMPS=$O/gaps_stamps.csv timeout -k 10 200 python tools/seal_gaps.py > $O/gaps.log 2>&1 || exit 1
DB=/tmp/pdb_r05u8_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
PDB_SEAL_STAMPS=$O/engine_stamps.csv timeout -k 10 300 integration/_build/pdb_dbbench_gpu_table --benchmarks=fillrandom \
  --num=10000000 --value_size=1024 --db=$DB/x > $O/fill.log 2>&1
