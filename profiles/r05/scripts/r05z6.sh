# round 5 shipped library (long-block CRCs written straight to pinned memory): GPU suite, smoke, the
# driver's line, then the engine's 10 M fill under rocprofv3 --kernel-trace --stats
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_run.sh r05z6 tests smoke bench_driver || exit 1
O=gpurun_out/r05z6_engine; mkdir -p $O
DB=/tmp/pdb_r05z6_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -- integration/_build/pdb_dbbench_gpu_table \
  --benchmarks=fillrandom --num=10000000 --value_size=1024 --db=$DB/x > $O/fill.log 2>&1
