#!/bin/bash
# Round 5, session g: offset/length batches (per-run flags + deferred pass): runs x residency grid on
# the NIC-ring layouts, the strided ring plans at each residency, and a kernel trace of the default
# offset/length batches (stream kernel vs deferred pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5g}
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ring_layouts.py > $O/${T}_ring_tests.log 2>&1 || { tail -40 $O/${T}_ring_tests.log; exit 1; }
tail -1 $O/${T}_ring_tests.log
RING_VARIANTS=offlengrid timeout -k 10 500 python -u tools/ring_probe.py > $O/${T}_ring_probe_grid.jsonl 2> $O/${T}_ring_probe_grid.err \
  || { tail $O/${T}_ring_probe_grid.err; exit 1; }
python3 - $O/${T}_ring_probe_grid.jsonl <<'PY'
import json, sys
rows = {}
for l in open(sys.argv[1]):
    d = json.loads(l)
    rows.setdefault((d['layout'], d['op']), []).append((d['ms'], d['form']))
for k, v in rows.items():
    v.sort()
    print(k, ' '.join(f"{f}={m:.4f}" for m, f in v))
PY
( cd /tmp && RING_VARIANTS=offlen timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_offlen_trace -o offlen \
    --output-format csv -- python3 $OLDPWD/tools/ring_probe.py template ring > $O/${T}_offlen_trace.log 2>&1 ) \
  || { tail $O/${T}_offlen_trace.log; exit 1; }
python3 - $O/${T}_offlen_trace/offlen_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'pkt_' in r['Name']:
        print(r['Name'][40:120], r['Calls'], r['AverageNs'], r['MinNs'])
PY
echo "session $T done"
