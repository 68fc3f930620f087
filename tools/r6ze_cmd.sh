#!/bin/bash
# Round 6, session ZE: C2 in the dispatch block order (the packet kernels' default) x run length x touch x residency.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6ze}
O=$R/gpurun_out; mkdir -p $O
for p in 1 2; do
  for c in ${CONFIGS:-c2 rx c2.x0 c2.s8.w0.x0 c2.s8.w0.t2.x0 c2.s8.w0.t0.x0 c2.t2.x0 c2.g0 c2.x0.g0 c2.s8.w0.x0.g0 c2.x256 c2}; do
    echo "== $c" >> $O/${T}_runs.log
    timeout -k 10 120 python tools/run_config.py $c 100 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
  done
done
grep "==\|ms=" $O/${T}_runs.log | paste - - | awk '{print $2, $(NF-4)}'
echo "session $T done"
