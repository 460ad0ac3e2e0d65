# round 5: phase stamps of every zero-copy seal (PDB_SEAL_STAMPS): the engine's 10 M fill against
# tools/seal_batches.py in isolation
set -o pipefail
O=gpurun_out/r05u5; mkdir -p $O
DB=/tmp/pdb_r05u5_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
PDB_SEAL_STAMPS=$O/engine_stamps.csv timeout -k 10 300 integration/_build/pdb_dbbench_gpu_table --benchmarks=fillrandom \
  --num=10000000 --value_size=1024 --db=$DB/x > $O/fill.log 2>&1 || exit 1
PDB_SEAL_STAMPS=$O/iso_stamps.csv timeout -k 10 300 python tools/seal_batches.py 1,4,16 > $O/iso.log 2>&1
