#!/bin/bash
# Round 6, session ZL: does C2's pseudo-header stream (12 B per segment, a separate array read with the
# plain policy, lines shared by neighbouring waves) cause its extra L2 tag stalls? C2 with and without
# it, and Rx, interleaved, then the tag-stall pass (tools/r6zj_cmd.sh) for the three.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6zl}
O=$R/gpurun_out; mkdir -p $O
for p in 1 2 3; do
  for c in ${CONFIGS:-c2 c2np rx}; do
    echo "== $c" >> $O/${T}_runs.log
    timeout -k 10 120 python tools/run_config.py $c 100 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
  done
done
grep "==\|ms=" $O/${T}_runs.log | paste - - | awk '{print $2, $(NF-4)}'
CONFIGS="c2 c2np rx" bash tools/r6zj_cmd.sh ${T}pmc 2>&1 | grep -v "rocclr\|direct_copy\|array<" | tail -7
echo "session $T done"
