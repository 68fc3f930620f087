#!/bin/bash
# Round 6, session ZO: C2 and the C5 shard at runs of 9-14 segments x 5-6 waves per SIMD against the default (16 at 5), three passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6zo}
O=$R/gpurun_out; mkdir -p $O
for p in 1 2 3; do
  for c in ${CONFIGS:-c2 c2.s10.w6 c2.s9.w6 c2.s11.w6 c2.s10.w5 c2.s10 c2.s14.w6 c2.w6 c5 c5.s10.w6 c5.s11.w6}; do
    echo "== $c" >> $O/${T}_runs.log
    timeout -k 10 120 python tools/run_config.py $c 100 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
  done
done
grep "==\|ms=" $O/${T}_runs.log | paste - - | awk '{print $2, $(NF-4)}'
echo "session $T done"
