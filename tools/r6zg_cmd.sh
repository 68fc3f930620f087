#!/bin/bash
# Round 6, session ZG: the mixed ring (40 / 576 / 1500-B frames in 1520-B slots) in live runs longer than
# the plan's 32 — up to the 63-KiB reach (42 slots) — Rx and Tx, interleaved, two passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6zg}
O=$R/gpurun_out; mkdir -p $O
for p in 1 2; do
  for c in ${CONFIGS:-rx_ring rx_ring.b2.s32 rx_ring.b2.s36 rx_ring.b2.s40 rx_ring.b2.s42 tx_ring tx_ring.b2.s40 rx_ringv rx_ringv.b2.s40 rx_nb2k.b2.s8 rx_nb2k.b2.s16 rx_nb2k.b2.s24}; do
    echo "== $c" >> $O/${T}_runs.log
    timeout -k 10 120 python tools/run_config.py $c 100 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
  done
done
grep "==\|ms=" $O/${T}_runs.log | paste - - | awk '{print $2, $(NF-4), $(NF-7), $(NF-6)}'
echo "session $T done"
