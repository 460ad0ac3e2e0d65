# round 5 final tree: GPU suite, smoke, the driver's line
set -o pipefail
bash tools/gpu_run.sh r05z7 tests smoke bench_driver
