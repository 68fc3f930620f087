#!/bin/bash
# Live segment stream run lengths 24-40 on the mixed pools (the plan's runs of 32 / 30 against longer
# ones within the reach), after the pseudo-header loads moved beside the descriptor loads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r5ac}
O=gpurun_out; mkdir -p $O
POOL_LIVE=1 timeout -k 10 400 python -u tools/varlen_pool_probe.py pool1520mix pool2kmix pool1520 > $O/${T}_varlen_pool_probe.jsonl \
  2> $O/${T}_varlen_pool_probe.err || { tail $O/${T}_varlen_pool_probe.err; exit 1; }
python3 - $O/${T}_varlen_pool_probe.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["layout"], d["form"], d["ms"], d["kernel"][:90])
PY
echo "session $T done"
