# round 5: zero-copy seals from pinned staging -- the table tests, the seal forms per batch size,
# then the engine's fillrandom 10M (BASELINE config 5) at 4 and 16 MiB seal batches
set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
DB=/tmp/pdb_r05l_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
timeout -k 10 300 python -u -m pytest tests/test_table.py tests/test_sst_files.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/seal_batches.py 4,16,32 > $O/seal_batches.log 2>&1 || exit 1
B=integration/_build
for mb in 4 16; do
  PDB_SEAL_BATCH_BYTES=$((mb << 20)) timeout -k 10 400 $B/pdb_dbbench_gpu_table --benchmarks=fillrandom --num=10000000 \
    --value_size=1024 --db=$DB/seal$mb > $O/fill_gpu_table_${mb}m.log 2>&1 || exit 1
  rm -rf $DB/seal$mb
done
grep -h "micros/op\|seal_copy" $O/*.log | cut -c1-400
