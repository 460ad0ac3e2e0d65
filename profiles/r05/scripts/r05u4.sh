# round 5: the engine's seal calls by batch size (C5 fillrandom 10 M, gpu_table), zero-copy default
set -o pipefail
O=gpurun_out/r05u4; mkdir -p $O
DB=/tmp/pdb_r05u4_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
timeout -k 10 300 integration/_build/pdb_dbbench_gpu_table --benchmarks=fillrandom --num=10000000 --value_size=1024 \
  --db=$DB/x > $O/fill_by_size.log 2>&1
grep -a '^{' $O/fill_by_size.log | cut -c1-300
