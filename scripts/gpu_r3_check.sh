#!/bin/bash
# New-kernel tests first, then the whole GPU suite, then env A/Bs.  A test step that
# ends other than pass / assertion failure (fault, abort, time limit) stops the script.
mkdir -p gpurun_out
step() {   # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step tfused 400 python -u -m pytest tests/test_gpu_tconv_fused.py ${EXTRA_TESTS:-} -v --timeout 120 --timeout-method thread
if [ "${FULL:-1}" = 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
fi
for ab in ${AB:-}; do
  k=${ab%%=*}; vals=${ab#*=}
  bash scripts/gpu_ab_env.sh "$k" ${vals//,/ } 3 || exit $?
done
