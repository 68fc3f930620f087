#!/bin/bash
# Round 6, session ZN: C2 run length x residency around runs of 8-16 at 6-7 waves per SIMD, three passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6zn}
O=$R/gpurun_out; mkdir -p $O
for p in 1 2 3; do
  for c in ${CONFIGS:-c2 c2.s8.w7 c2.s10.w7 c2.s12.w7 c2.w7 c2.s12.w6 c2.s8.w6 c2.s10.w6 c2.s20 c2.s20.w6}; do
    echo "== $c" >> $O/${T}_runs.log
    timeout -k 10 120 python tools/run_config.py $c 100 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
  done
done
grep "==\|ms=" $O/${T}_runs.log | paste - - | awk '{print $2, $(NF-4)}'
echo "session $T done"
