#!/bin/bash
# Round 6, session O: the C5 shard's block order against its allocation — the kernel in the slice,
# dispatch and chunked orders, the read probe in the dispatch and slice orders, on the first allocation
# and on a second one (a box where the first allocation is slow is the one this is for).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6o}
O=$R/gpurun_out; mkdir -p $O
C5P_VARIANTS=${C5P_VARIANTS:-c5_kernel,c5_xcd0,c5_x64,c5_x256,c5_touch0,c5_run_probe,c5_run_probe_x1,alloc2,alloc2_xcd0,alloc2_run_probe,alloc2_run_probe_x1} \
  timeout -k 10 500 python -u tools/c5_probe.py > $O/${T}_c5_probe.jsonl 2> $O/${T}_c5_probe.err || { tail $O/${T}_c5_probe.err; exit 1; }
cut -c1-200 $O/${T}_c5_probe.jsonl
echo "session $T done"
