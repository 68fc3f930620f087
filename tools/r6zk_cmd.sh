#!/bin/bash
# Round 6, session ZK: the dense segment stream's row touch without the pieces already in flight
# (NETCSUM_TUNE_STREAM_TOUCH 2: the first D pieces' touches collide with their own pending stream
# misses in the L2) against the default touch, C2 and the C5 shard, interleaved; parity of every touch
# mode first; then the L2 tag-stall pass for both.
# EXPERIMENT BUILD (touch mode 2 in seg_stream_kernel, parity-tested, then reverted: slower, more tag
# stalls, profiles/r6zk_touch_runs.log, r6zk_pmc.json); on the committed sources TUNE_STREAM_TOUCH is -1..1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6zk}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k touch_and_residency -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
for p in 1 2 3; do
  for c in ${CONFIGS:-c2 c2.t2 rx c5 c5.t2}; do
    echo "== $c" >> $O/${T}_runs.log
    timeout -k 10 120 python tools/run_config.py $c 100 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
  done
done
grep "==\|ms=" $O/${T}_runs.log | paste - - | awk '{print $2, $(NF-4)}'
CONFIGS="c2 c2.t2" bash tools/r6zj_cmd.sh ${T}pmc 2>&1 | grep -v "_p2" | tail -4
echo "session $T done"
