#!/bin/bash
# Round 6, session ZM: the packed Rx kernel at capped residencies (4 / 5 / 6 / 8 waves per SIMD) beside C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6zm}
O=$R/gpurun_out; mkdir -p $O
for p in 1 2 3; do
  for c in ${CONFIGS:-c2 rx rx.w4 rx.w5 rx.w6 rx.w8 c2np.w0 c2np.s8.w0}; do
    echo "== $c" >> $O/${T}_runs.log
    timeout -k 10 120 python tools/run_config.py $c 100 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
  done
done
grep "==\|ms=" $O/${T}_runs.log | paste - - | awk '{print $2, $(NF-4)}'
echo "session $T done"
