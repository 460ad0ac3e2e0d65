# round 5 closing library: GPU suite, smoke, the driver's bench line, every row's 50-step line
set -o pipefail
bash tools/gpu_run.sh r05y tests smoke bench_driver bench_rows
