# round 5: A/B of the long-block split in the engine (10 M fills, one box): split / none / none / split
set -o pipefail
O=gpurun_out/r05ub; mkdir -p $O
DB=/tmp/pdb_r05ub_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
fill() {  # name env...
  local name=$1; shift
  rm -rf $DB/x
  env "$@" timeout -k 10 300 integration/_build/pdb_dbbench_gpu_table --benchmarks=fillrandom --num=10000000 \
    --value_size=1024 --db=$DB/x > $O/$name.log 2>&1 || return 1
  grep -a "micros/op" $O/$name.log | head -1
}
fill split_a PDB_X=1 && fill none_a PDB_LONG_BLOCK=0 && fill none_b PDB_LONG_BLOCK=0 && fill split_b PDB_X=1
