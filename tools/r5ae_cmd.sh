#!/bin/bash
# Live kernels at 8 waves per SIMD (their rare fallbacks one chunk per lane at a time): the pool probe
# and floors (tools/r5y_cmd.sh), then the chain tests and the chain row by events in the tiled groups
# (default) and the live pass 1 (TUNE_KERNEL 3) at runs of 8 / 16 / 24 and depth 4 / 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r5ae}
O=gpurun_out; mkdir -p $O
bash tools/r5y_cmd.sh $T || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_chains.py \
  > $O/${T}_chain_tests.log 2>&1 || { tail -40 $O/${T}_chain_tests.log; exit 1; }
tail -1 $O/${T}_chain_tests.log
for r in 1 2; do
for c in chains chains.k3 chains.k3.s8 chains.k3.s8.d4 chains.k3.d4 chains.k3.s24 chains.k3.s24.d4; do
  timeout -k 10 120 python -u tools/run_config.py $c 200 2>/dev/null >> $O/${T}_chains.log || { tail $O/${T}_chains.log; exit 1; }
done
done
cat $O/${T}_chains.log
echo "session $T done"
