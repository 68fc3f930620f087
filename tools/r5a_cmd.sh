#!/bin/bash
# Round 5, session a: the shared-hardware-queue burst server test against round 4's library (the
# "before" record; failures expected, the run must only end normally) and against the new sources,
# then the burst tests and the whole -m gpu suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5a}
O=gpurun_out; mkdir -p $O
REC=$O/${T}_burst_server_queue.jsonl
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
NETCSUM_LIB=$PWD/uc-tcp-ip_amd/build/libnetcsum_r4base.so NETCSUM_BURST_SERVER_RECORD=$REC \
  timeout -k 10 150 $PYT tests/test_gpu_burst_server.py > $O/${T}_r4base_queue.log 2>&1
rc=$?; echo "round-4 library: rc=$rc"; tail -3 $O/${T}_r4base_queue.log
[ $rc -le 1 ] || exit 1                                      # only a pass or a failed assertion goes on
NETCSUM_BURST_SERVER_RECORD=$REC timeout -k 10 150 $PYT tests/test_gpu_burst_server.py > $O/${T}_queue.log 2>&1 \
  || { tail -30 $O/${T}_queue.log; exit 1; }
tail -2 $O/${T}_queue.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/${T}_gpu_tests.log 2>&1 || { tail -40 $O/${T}_gpu_tests.log; exit 1; }
tail -2 $O/${T}_gpu_tests.log
cat $REC
echo "session $T done"
