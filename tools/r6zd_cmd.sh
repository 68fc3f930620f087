#!/bin/bash
# Round 6, session ZD: C2 with segment-start window touches (NETCSUM_TUNE_STREAM_TOUCH 2 / 3 / 4: the
# Rx prologue's 96-B plain loads per datagram, awaited / 32 B awaited / 96 B retired after the stream)
# against the 1-KiB row touch, interleaved with rx; parity of every touch mode first.
# EXPERIMENT BUILD (touch modes 2-4 in seg_stream_kernel, parity-tested, then reverted: slower than the
# row touch, profiles/r6zd_c2_runs.log); on the committed sources TUNE_STREAM_TOUCH accepts -1..1 only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6zd}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k touch_and_residency -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
for p in 1 2; do
  for c in ${CONFIGS:-c2 rx c2.t2 c2.t3 c2.t4 c2.t2.w0 c2.t2.s8.w0 c2.t2.s8.w7 c2.t2.w6 c2.t2.s12 c2.t0 c2}; do
    echo "== $c" >> $O/${T}_runs.log
    timeout -k 10 120 python tools/run_config.py $c 100 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
  done
done
grep "==\|ms=" $O/${T}_runs.log | paste - - | awk '{print $2, $(NF-4)}'
echo "session $T done"
