#!/bin/bash
# Chain pass 1 in the live-sector stream (chain_live_piece_kernel): the chain GPU tests, then the chain
# row by events in the default form, runs of 8 / 32 pieces, and round 4's tiled groups (TUNE_KERNEL 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r5u}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chains.py \
  tests/test_gpu_threads.py > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
for r in 1 2; do
for c in chains chains.k2 chains.s8 chains.s8.d4 chains.s16.d4 chains.s24 chains.s24.d4 chains.s12; do
  timeout -k 10 120 python -u tools/run_config.py $c 200 >> $O/${T}_chains.log 2>&1 || { tail $O/${T}_chains.log; exit 1; }
done
done
cat $O/${T}_chains.log
echo "session $T done"
