# round 5: the engine (BASELINE config 5) -- copy-inclusive seal rate in fillrandom 10M at 4 / 16 /
# 32 MiB seal batches (pinned staging), one run with the engine's destructor (--close_db=1), then
# verified readrandom at 1/2/4/8/16 threads on the GPU and CPU builds over one 10M database
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
DB=/tmp/pdb_r05d_$$; mkdir -p $DB; trap 'rm -rf $DB' EXIT
df -h /tmp | tail -1 > $O/disk.txt
B=integration/_build
for mb in 4 16 32; do
  PDB_SEAL_BATCH_BYTES=$((mb << 20)) timeout -k 10 400 $B/pdb_dbbench_gpu_table --benchmarks=fillrandom --num=10000000 \
    --value_size=1024 --db=$DB/seal$mb > $O/fill_gpu_table_${mb}m.log 2>&1 || exit 1
  [ $mb = 32 ] || rm -rf $DB/seal$mb
done
# the last database (32 MiB batches) is the readrandom database; one more fill with the destructor
timeout -k 10 400 $B/pdb_dbbench_gpu_table --benchmarks=fillrandom --num=1000000 --value_size=1024 --close_db=1 \
  --db=$DB/close > $O/fill_gpu_table_1m_close_db.log 2>&1 || exit 1
rm -rf $DB/close
for v in gpu_table cpu; do
  for t in 1 2 4 8 16; do
    timeout -k 10 300 $B/pdb_dbbench_$v --benchmarks=readrandom --use_existing_db=1 --num=10000000 --reads=500000 \
      --threads=$t --value_size=1024 --verify_checksums=1 --db=$DB/seal32 > $O/read_${v}_t$t.log 2>&1 || exit 1
  done
done
grep -h "micros/op\|seal_copy" $O/*.log | cut -c1-300
