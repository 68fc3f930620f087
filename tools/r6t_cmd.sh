#!/bin/bash
# Round 6, session T: chain pass 1 with the row touch of a group's first pieces (.t1) against none.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6t}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chains.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
for c in ${CONFIGS:-chains chains.t1 chains chains.t1 chains chains.t1}; do
  echo "== $c" >> $O/${T}_runs.log
  timeout -k 10 120 python tools/run_config.py $c 60 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
done
grep "==\|ms=" $O/${T}_runs.log | cut -c1-160
echo "session $T done"
