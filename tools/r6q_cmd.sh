#!/bin/bash
# Round 6, session Q: strided batches in XCD chunks of 256 blocks by default — parity, C2 / C5 / C3 /
# ring-shaped strided batches against the one-slice order (.x1), chain pass 1 in chunked tile orders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6q}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chains.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
for c in ${CONFIGS:-c5 c5.x1 c2 c2.x1 chains chains.x0 chains.x64 chains.x256 c5 c5.x1 c2 c2.x1 chains chains.x0 chains.x64 chains.x256}; do
  echo "== $c" >> $O/${T}_runs.log
  timeout -k 10 120 python tools/run_config.py $c 40 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
done
grep "==\|ms=" $O/${T}_runs.log | cut -c1-160
echo "session $T done"
