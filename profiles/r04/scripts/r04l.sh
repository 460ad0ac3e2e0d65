# round 4: where the record kernel's waves wait -- shipped (0), bank-class rotation (169), mask selects (172)
set -o pipefail
PMC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
  timeout -k 10 900 bash tools/span_pmc.sh r04l_wait 0,169,172 wal1000,wal400 > gpurun_out/r04l.log 2>&1; rc=$?; tail -1 gpurun_out/r04l.log; exit $rc
