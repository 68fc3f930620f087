#!/bin/bash
# Round 6, session ZH: the 20 / 556 / 1480-B pool mix in 1520-B buffers: run length, depth, residency.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6zh}
O=$R/gpurun_out; mkdir -p $O
for p in 1 2; do
  for c in ${CONFIGS:-pool1520mix pool1520mix.s16 pool1520mix.s24 pool1520mix.s32 pool1520mix.d8 pool1520mix.s24.d8 pool1520mix.w6 pool1520mix.w8 pool1520mix.lc0 pool2kmix pool2kmix.s16 pool2kmix.d4}; do
    echo "== $c" >> $O/${T}_runs.log
    timeout -k 10 120 python tools/run_config.py $c 100 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
  done
done
grep "==\|ms=" $O/${T}_runs.log | paste - - | awk '{print $2, $(NF-4), $(NF-7), $(NF-6)}'
echo "session $T done"
