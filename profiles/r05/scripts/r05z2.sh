# round 5 closing library (long-block split in the zero-copy host path): GPU suite, smoke, driver line
set -o pipefail
bash tools/gpu_run.sh r05z2 tests smoke bench_driver
