# round 5 final on-disk libraries (relinked by build()): GPU suite, smoke, the driver's line
set -o pipefail
bash tools/gpu_run.sh r05z9 tests smoke bench_driver
