#!/bin/bash
# Round 5, session l: varlen pool plans (pipe 16x6 / 8x8): tests and the pool probe on every layout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5l}
O=$PWD/gpurun_out; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PYT tests/test_gpu_varlen_pool.py tests/test_gpu_parity.py tests/test_gpu_configs_full.py > $O/${T}_varlen_tests.log 2>&1 \
  || { tail -40 $O/${T}_varlen_tests.log; exit 1; }
tail -1 $O/${T}_varlen_tests.log
POOL_PIPES=1 timeout -k 10 500 python -u tools/varlen_pool_probe.py > $O/${T}_varlen_pool_probe.jsonl 2> $O/${T}_varlen_pool_probe.err \
  || { tail $O/${T}_varlen_pool_probe.err; exit 1; }
python3 - $O/${T}_varlen_pool_probe.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f"{d['layout']:12s} {d['form']:12s} {d['ms']:.4f} {d['frac_of_8TBps']:.3f} {d.get('parity_sample_ok', '')} {d['kernel'][:90]}")
PY
echo "session $T done"
