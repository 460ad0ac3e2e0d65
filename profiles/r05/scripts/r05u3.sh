# round 5: the zero-copy seal of a 16-MiB pinned batch under host-memory load (0..12 threads copying)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/seal_batches.py 16 -1 0,2,4,8,12 > gpurun_out/r05u3_seal_hostload.log 2>&1
