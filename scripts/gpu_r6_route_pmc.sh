#!/bin/bash
# Round 6: HBM bytes of the skip-half data gradient variants (scripts/route_micro.py), one
# counter pass each (FETCH_SIZE, then WRITE_SIZE), per dispatch.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6routepmc; mkdir -p $o
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/fetch -o run -- python scripts/route_micro.py 2 > $o/fetch.log 2>&1 || { echo "fetch rc=$?"; tail $o/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/write -o run -- python scripts/route_micro.py 2 > $o/write.log 2>&1 || { echo "write rc=$?"; tail $o/write.log; exit 1; }
find $o -name "*counter_collection.csv" | head
