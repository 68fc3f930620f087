#!/bin/bash
# Round 6, session ZA: why the packed Rx kernel (runs of 8 datagrams, header-window touch) streams
# the same 1 M x 1500 B faster per byte than C2's segment stream (runs of 16, 1-KiB row touch):
# C2 run lengths x touch x residency, interleaved with rx, two passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6za}
O=$R/gpurun_out; mkdir -p $O
for p in 1 2; do
  for c in ${CONFIGS:-c2 rx c2.s8 c2.s8.t0 c2.s8.w0 c2.s12 c2.s32 c2.w4 c2.w6 c2.nt0 rx.t1 c2}; do
    echo "== $c" >> $O/${T}_runs.log
    timeout -k 10 120 python tools/run_config.py $c 100 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
  done
done
grep "==\|ms=" $O/${T}_runs.log | cut -c1-220
echo "session $T done"
