#!/bin/bash
# Round 6: new / changed kernel tests (bounds sentinels, conv_dw, tconv segmented rows).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6t; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bounds.py \
  tests/test_gpu_conv_dw.py "tests/test_gpu_kernels.py::test_tconv_fwd_shuffle_and_dgrad" > $o/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -3 $o/tests.log
