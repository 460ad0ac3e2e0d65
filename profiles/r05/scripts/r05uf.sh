# round 5: the engine's 10 M fill under rocprofv3 --kernel-trace --stats with the long-block split
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05uf; mkdir -p $O
DB=/tmp/pdb_r05uf_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -- integration/_build/pdb_dbbench_gpu_table \
  --benchmarks=fillrandom --num=10000000 --value_size=1024 --db=$DB/x > $O/fill.log 2>&1
