#!/bin/bash
# Round 5, session b: the device-chosen packet plan (TUNE_PKT_BOUND 4) — ring-layout parity tests,
# then the NIC-ring probe of the plan against the fixed forms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5b}
O=gpurun_out; mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ring_layouts.py > $O/${T}_ring_tests.log 2>&1 || { tail -40 $O/${T}_ring_tests.log; exit 1; }
tail -2 $O/${T}_ring_tests.log
RING_VARIANTS=plan timeout -k 10 500 python -u tools/ring_probe.py > $O/${T}_ring_probe_plan.jsonl 2> $O/${T}_ring_probe_plan.err \
  || { tail $O/${T}_ring_probe_plan.err; exit 1; }
python3 - $O/${T}_ring_probe_plan.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f"{d['layout']:9s} {d['form']:16s} {d['op']} {d['ms']:.4f} {d.get('plan', '')}")
PY
echo "session $T done"
