#!/bin/bash
# Round 6, session G: the C5 shard's per-GPU deficit, continued — pieces in flight and residency
# (tools/c5_probe.py d6 / d8 / w4 / w6 / w8) against the kernel and its read probe, C5 and C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6g}
O=$R/gpurun_out; mkdir -p $O
C5P_VARIANTS=kernel,run_probe,d6,d8,w4,w6,w8 timeout -k 10 400 python -u tools/c5_probe.py > $O/${T}_c5_probe.jsonl 2> $O/${T}_c5_probe.err \
  || { tail $O/${T}_c5_probe.err; exit 1; }
cat $O/${T}_c5_probe.jsonl
echo "session $T done"
