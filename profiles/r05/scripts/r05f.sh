set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 300 python tools/debug_concurrent.py 20 > $O/debug.log 2>&1; echo rc=$?
tail -30 $O/debug.log
