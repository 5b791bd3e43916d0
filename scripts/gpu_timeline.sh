#!/bin/bash
# One-step kernel timelines (tools/timeline.py) of the headline bench and the
# normalised configs, plus their bench lines.
#   bash scripts/gpu_timeline.sh <tag> [extra bench args ...]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-cur}; shift
o=gpurun_out/tl_$tag
rm -rf $o; mkdir -p $o
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $o/$n -o run -- \
    python bench.py --steps 4 --warmup 2 "$@" > $o/$n.log 2>&1 || return $?
  local f=$(find $o/$n -name "*kernel_trace.csv" | head -1)
  python tools/timeline.py $f "$n: bench.py $*" > $o/$n.md || return $?
  head -22 $o/$n.md
}
run plain "$@" && \
run bn --norm batch "$@" && \
run gn16 --norm group --dtype fp16 "$@"
