# round 5 final library: GPU suite, smoke, the driver's line, and one stamped 10 M fill
set -o pipefail
bash tools/gpu_run.sh r05z5 tests smoke bench_driver || exit 1
O=gpurun_out/r05z5_engine; mkdir -p $O
DB=/tmp/pdb_r05z5_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
PDB_SEAL_STAMPS=$O/engine_stamps.csv timeout -k 10 300 integration/_build/pdb_dbbench_gpu_table --benchmarks=fillrandom \
  --num=10000000 --value_size=1024 --db=$DB/x > $O/fill.log 2>&1
