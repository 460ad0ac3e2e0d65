# round 5 final tree: every row's 50-step bench line once more
set -o pipefail
bash tools/gpu_run.sh r05z8 bench_rows
