#!/bin/bash
# Round 5, session j: varlen pool plans (the lane-group pipe form for gapped long segments): tests,
# the pool probe (default = the plan, fixed forms, residency), then the whole -m gpu suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5j}
O=$PWD/gpurun_out; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PYT tests/test_gpu_varlen_pool.py > $O/${T}_varlen_tests.log 2>&1 || { tail -40 $O/${T}_varlen_tests.log; exit 1; }
tail -1 $O/${T}_varlen_tests.log
timeout -k 10 400 python -u tools/varlen_pool_probe.py > $O/${T}_varlen_pool_probe.jsonl 2> $O/${T}_varlen_pool_probe.err \
  || { tail $O/${T}_varlen_pool_probe.err; exit 1; }
python3 - $O/${T}_varlen_pool_probe.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f"{d['layout']:12s} {d['form']:8s} {d['ms']:.4f} {d['frac_of_8TBps']:.3f} {d.get('parity_sample_ok', '')} {d['kernel'][:90]}")
PY
timeout -k 10 900 $PYT -m gpu tests > $O/${T}_gpu_tests.log 2>&1 || { tail -40 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
echo "session $T done"
