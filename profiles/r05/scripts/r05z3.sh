# round 5 shipped library: GPU suite, smoke, the driver's line, then BASELINE config 5 at 10 M
set -o pipefail
bash tools/gpu_run.sh r05z3 tests smoke bench_driver || exit 1
bash tools/c5_run.sh r05_c5c 10000000 "ref cpu gpu_table"
