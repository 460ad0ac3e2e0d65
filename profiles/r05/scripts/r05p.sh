# round 5 final kernels: rocprof + PMC traffic of the WAL rows and C2, then the record kernel's SQ counters
set -o pipefail
bash tools/gpu_run.sh r05p prof_wal counters_span
