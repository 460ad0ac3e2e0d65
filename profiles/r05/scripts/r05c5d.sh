# round 5: BASELINE config 5 at 10 M with the shipped library (reference db_bench, CPU build, GPU hooks)
set -o pipefail
bash tools/c5_run.sh r05_c5d 10000000 "ref cpu gpu_table"
