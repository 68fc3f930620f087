#!/bin/bash
# The live-sector stream for segments one per pool buffer (seg_live_varlen_kernel, plan 3): the varlen
# GPU tests, then the pool probe with the run-length x depth sweep (POOL_LIVE) beside the pipe form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r5s}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_varlen_pool.py \
  tests/test_gpu_parity.py tests/test_gpu_threads.py tests/test_gpu_configs_full.py > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
POOL_LIVE=1 timeout -k 10 400 python -u tools/varlen_pool_probe.py > $O/${T}_varlen_pool_probe.jsonl 2> $O/${T}_varlen_pool_probe.err \
  || { tail $O/${T}_varlen_pool_probe.err; exit 1; }
python3 - $O/${T}_varlen_pool_probe.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f"{d['layout']:12s} {d['form']:12s} {d['ms']:.4f} {d['frac_of_8TBps']:.3f} {d.get('parity_sample_ok', '')} {d['kernel'][:80]}")
PY
echo "session $T done"
