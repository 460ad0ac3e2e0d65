# round 5: the engine's 10 M fill with PDB_SEAL_STAMPS (bytes, blocks and the largest block per seal)
set -o pipefail
O=gpurun_out/r05u9; mkdir -p $O
DB=/tmp/pdb_r05u9_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
PDB_SEAL_STAMPS=$O/engine_stamps.csv timeout -k 10 300 integration/_build/pdb_dbbench_gpu_table --benchmarks=fillrandom \
  --num=10000000 --value_size=1024 --db=$DB/x > $O/fill.log 2>&1
