#!/bin/bash
# Round 6, session ZC: C2 in the Rx kernel's shape (runs of 8, no row touch, full residency) and neighbours.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6zc}
O=$R/gpurun_out; mkdir -p $O
for p in 1 2; do
  for c in ${CONFIGS:-c2 rx c2.s8.w0.t0 c2.w0.t0 c2.w0 c2.s8.w0 c2.s6.w0 c2.s10.w0 c2.s12.w0 c2.s8.w0.d6 c2.s8.w8 c2.s8.w7 c2}; do
    echo "== $c" >> $O/${T}_runs.log
    timeout -k 10 120 python tools/run_config.py $c 100 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
  done
done
grep "==\|ms=" $O/${T}_runs.log | cut -c1-220
echo "session $T done"
