#!/bin/bash
# Round 6, session V: chain pass 1 (one-record live stream) run-length / depth sweep, then the chain
# row's kernel trace + PMC (pass 1 and the combine separately) on the final form.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6v}
O=$R/gpurun_out; mkdir -p $O
for c in ${CONFIGS:-chains chains.s12 chains.s20 chains.s24 chains.s30 chains.d4 chains.s12.d4 chains.s24.d4 chains chains.s12 chains.s20 chains.s24 chains.s30 chains.d4 chains.k4}; do
  echo "== $c" >> $O/${T}_runs.log
  timeout -k 10 120 python tools/run_config.py $c 60 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
done
grep "==\|ms=" $O/${T}_runs.log | cut -c1-200
timeout -k 10 400 bash tools/gpu_pmc_all.sh ${T} chains || exit 1
echo "session $T done"
