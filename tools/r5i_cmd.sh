#!/bin/bash
# Round 5, session i: offset/length ring plans with the inline form for dense rings in order: the
# ring-layout tests and the NIC-ring probe (plan, fixed forms, offset/length).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5i}
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ring_layouts.py > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
RING_VARIANTS=plan timeout -k 10 400 python -u tools/ring_probe.py > $O/${T}_ring_probe.jsonl 2> $O/${T}_ring_probe.err \
  || { tail $O/${T}_ring_probe.err; exit 1; }
python3 - $O/${T}_ring_probe.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f"{d['layout']:9s} {d['form']:16s} {d['op']} {d['ms']:.4f} {d['kernel'][-60:]}")
PY
echo "session $T done"
