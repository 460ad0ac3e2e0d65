# round 5: the engine's seals by DMA from the reused page-locked batches (PDB_HOST_MAPPED=0) against
# zero-copy, C5 fillrandom 10 M; DMA in one group (16 MiB) and in 4-MiB groups (copies overlap kernels)
set -o pipefail
O=gpurun_out/r05u2; mkdir -p $O
DB=/tmp/pdb_r05u2_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
fill() {  # name env...
  local name=$1; shift
  rm -rf $DB/x
  env "$@" timeout -k 10 300 integration/_build/pdb_dbbench_gpu_table --benchmarks=fillrandom --num=10000000 \
    --value_size=1024 --db=$DB/x > $O/$name.log 2>&1 || return 1
  grep -a "micros/op" $O/$name.log | head -2
  grep -ao '"seal_[a-z_]*": [0-9.]*' $O/$name.log | tr '\n' ' '; echo
}
fill zero_copy PDB_X=1 && fill dma_16m PDB_HOST_MAPPED=0 && fill dma_4m PDB_HOST_MAPPED=0 PDB_HOST_CHUNK_BYTES=4194304 \
  && fill zero_copy2 PDB_X=1
