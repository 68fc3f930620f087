#!/bin/bash
# Round 6, sessions U / X: chain pass 1 as the segment live-sector stream with one record per piece
# (default, TUNE_KERNEL 5) against the tiled groups (.k4): runs (.sN), depth (.dN), compacted or not (.lcN).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6u}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_chains.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
for c in ${CONFIGS:-chains chains.k4 chains chains.k4 chains}; do
  echo "== $c" >> $O/${T}_runs.log
  timeout -k 10 120 python tools/run_config.py $c 60 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
done
grep "==\|ms=" $O/${T}_runs.log | cut -c1-200
echo "session $T done"
