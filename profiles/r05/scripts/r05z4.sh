# round 5 shipped library (long blocks split on both host routes): GPU suite, smoke, the driver's line
set -o pipefail
bash tools/gpu_run.sh r05z4 tests smoke bench_driver
