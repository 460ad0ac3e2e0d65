# round 5: the verify's ok bytes through the LDS ring -- parity, the bench line, rocprof + WRITE_SIZE
set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sst4k.py tests/test_sst_files.py tests/test_table.py tests/test_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload sst_verify --no-copy-inclusive --steps 50 > $O/bench_sst_verify.log 2>&1 || exit 1
timeout -k 10 900 bash tools/profile.sh r05m_prof_sst_verify sst_verify > $O/prof.log 2>&1 || exit 1
tail -3 $O/tests.log; grep -v amdgpu $O/bench_sst_verify.log | cut -c1-600; tail -5 $O/prof.log
