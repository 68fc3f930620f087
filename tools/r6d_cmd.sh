#!/bin/bash
# Round 6, session D: the compacted pool kernel's run length x depth sweep (POOL_LIVE), all four layouts.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6d}
O=$R/gpurun_out; mkdir -p $O
POOL_LIVE=1 timeout -k 10 500 python -u tools/varlen_pool_probe.py pool1520mix pool2kmix pool1520 pool2k > $O/${T}_varlen_pool_sweep.jsonl \
  2> $O/${T}_varlen_pool_sweep.err || { tail $O/${T}_varlen_pool_sweep.err; exit 1; }
python3 -c "
import json
for l in open('$O/${T}_varlen_pool_sweep.jsonl'):
    d=json.loads(l); print(d['layout'], d['form'], d['ms'], d['kernel'][:60])"
echo "session $T done"
