# round 5: the engine's seals by batch size, DMA route (PDB_HOST_MAPPED=0) against zero-copy
set -o pipefail
O=gpurun_out/r05u6; mkdir -p $O
DB=/tmp/pdb_r05u6_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
fill() {  # name env...
  local name=$1; shift
  rm -rf $DB/x
  env "$@" timeout -k 10 300 integration/_build/pdb_dbbench_gpu_table --benchmarks=fillrandom --num=10000000 \
    --value_size=1024 --db=$DB/x > $O/$name.log 2>&1 || return 1
}
fill dma PDB_HOST_MAPPED=0 && fill zero_copy PDB_X=1
