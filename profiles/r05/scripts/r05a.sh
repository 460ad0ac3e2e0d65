set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit 1
for w in wal100 wal400 wal1000 wal; do
  timeout -k 10 200 python bench.py --workload $w --no-copy-inclusive --no-cpu-baseline --steps 50 > $O/bench_$w.log 2>&1 || exit 1
done
timeout -k 10 300 python tools/ab_span.py 0,63,64,67 wal1000,wal100 4 > $O/ab_parts.log 2>&1 || exit 1
