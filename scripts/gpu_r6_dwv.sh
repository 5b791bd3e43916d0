#!/bin/bash
# conv_dw operand sources, isolated launches at the benched shape (scripts/dw_micro.py).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6dwv; mkdir -p $o
timeout -k 10 120 python scripts/dw_micro.py 1024 10 > $o/micro.md 2>&1 || { echo "micro rc=$?"; tail $o/micro.md; exit 1; }
cat $o/micro.md
