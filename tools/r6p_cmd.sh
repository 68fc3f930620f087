#!/bin/bash
# Round 6, session P: the chunk size of the XCD block order (NETCSUM_TUNE_STREAM_XCD C) on C5 and C2,
# against the one-slice order and the read probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6p}
O=$R/gpurun_out; mkdir -p $O
C5P_VARIANTS=${C5P_VARIANTS:-_xcd1,_x16,_x64,_x128,_x256,_x1024,_x4096,_xcd0,_run_probe,_run_probe_x1,_run_probe_x256} \
  timeout -k 10 500 python -u tools/c5_probe.py > $O/${T}_c5_probe.jsonl 2> $O/${T}_c5_probe.err || { tail $O/${T}_c5_probe.err; exit 1; }
cut -c1-200 $O/${T}_c5_probe.jsonl
echo "session $T done"
