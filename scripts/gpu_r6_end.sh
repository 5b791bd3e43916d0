#!/bin/bash
# Round 6 end: whole GPU suite + smoke, then every BASELINE config once more.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6end; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_suite.log 2>&1 || { echo "suite rc=$?"; tail -40 $o/gpu_suite.log; exit 1; }
tail -2 $o/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
SKIP_FP32=1 bash scripts/gpu_r6_configs.sh "64" "8 16"
