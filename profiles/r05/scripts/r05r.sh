# round 5: finer tail split A/B (variant 187), then BASELINE config 5 at 10 M on one box (reference db_bench,
# the engine as shipped, the GPU hooks)
set -o pipefail
AB_VARIANTS=0,187 AB_WL=wal100,wal400,wal1000,wal AB_ROUNDS=6 bash tools/gpu_run.sh r05r ab_vs || exit 1
bash tools/c5_run.sh r05_c5 10000000 "ref cpu gpu_table" fillrandom,readrandom 1
