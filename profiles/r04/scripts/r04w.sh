# round 4 (late): scalar server with two polls in flight -- server tests, then the phase breakdown
set -o pipefail
O=gpurun_out/r04w; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_scalar_server.py tests/test_capi.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/scalar_phases.py $O/scalar_phases.json 20000 > $O/scalar_phases.log 2>&1 || { echo PHASES_FAILED; tail $O/scalar_phases.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/scalar_phases.json'))
for s,v in d['sizes'].items(): print(s, {k: (x['median'], x['min']) for k,x in v['us'].items()})"
