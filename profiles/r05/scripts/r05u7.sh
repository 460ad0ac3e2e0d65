# round 5: the engine's seals by batch size with the database on tmpfs (no block-device I/O) against
# the overlay disk, zero-copy default
set -o pipefail
O=gpurun_out/r05u7; mkdir -p $O
df -h /dev/shm /tmp | tee $O/df.txt
SHM=/dev/shm/pdb_r05u7_$$; DB=/tmp/pdb_r05u7_$$; mkdir -p $SHM $DB; trap 'rm -rf $SHM $DB' EXIT
fill() {  # name dir
  rm -rf $2/x
  timeout -k 10 300 integration/_build/pdb_dbbench_gpu_table --benchmarks=fillrandom --num=10000000 \
    --value_size=1024 --db=$2/x > $O/$1.log 2>&1 || return 1
  rm -rf $2/x
}
fill shm $SHM && fill disk $DB
