#!/bin/bash
# Round 6, session N: chain pass 1's balanced grid (NETCSUM_TUNE_CHAIN_GRID k) against its tiles, and the
# chunked XCD block order (NETCSUM_TUNE_STREAM_XCD C >= 2) — parity under every option, then the C5 shard on its first allocation (the slow one on slow boxes) and on a second one in
# the plain, slice and chunked orders, beside the read probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6n}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "touch_and_residency" > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_chains.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/${T}_chain_tests.log 2>&1 || { tail -30 $O/${T}_chain_tests.log; exit 1; }
tail -1 $O/${T}_chain_tests.log
for c in ${CHAINS:-chains chains.cg1 chains.cg2 chains.cg1.x1 chains.cg4 chains chains.cg1 chains.cg2 chains.cg1.x1 chains.cg4}; do
  timeout -k 10 120 python tools/run_config.py $c 40 >> $O/${T}_chains_runs.log 2>&1 || { tail $O/${T}_chains_runs.log; exit 1; }
done
grep "ms=" $O/${T}_chains_runs.log
C5P_VARIANTS=${C5P_VARIANTS:-kernel,xcd0,x4,x16,x64,x256,run_probe,alloc2,alloc2_xcd0,alloc2_x16} timeout -k 10 500 python -u tools/c5_probe.py \
  > $O/${T}_c5_probe.jsonl 2> $O/${T}_c5_probe.err || { tail $O/${T}_c5_probe.err; exit 1; }
cut -c1-200 $O/${T}_c5_probe.jsonl
echo "session $T done"
