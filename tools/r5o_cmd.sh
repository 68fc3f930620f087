#!/bin/bash
# Deferred offset/length pass in ordered sub-runs: the packet and ring-layout GPU tests, then the
# ring probe's offset/length variants on every layout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r5o}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ring_layouts.py tests/test_gpu_pktstream.py tests/test_gpu_varlen_pool.py > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -3 $O/${T}_tests.log
RING_VARIANTS=offlen timeout -k 10 400 python -u tools/ring_probe.py > $O/${T}_ring_probe_offlen.jsonl 2> $O/${T}_ring_probe.err || { tail $O/${T}_ring_probe.err; exit 1; }
timeout -k 10 400 python -u tools/ring_probe.py nb2k ring > $O/${T}_ring_probe.jsonl 2>> $O/${T}_ring_probe.err || { tail $O/${T}_ring_probe.err; exit 1; }
python3 -c "
import json
for f in ('$O/${T}_ring_probe_offlen.jsonl','$O/${T}_ring_probe.jsonl'):
    for l in open(f):
        try: d=json.loads(l)
        except Exception: continue
        print(d.get('layout'), d.get('variant'), d.get('ms'), d.get('kernel'))
"
echo "session $T done"
