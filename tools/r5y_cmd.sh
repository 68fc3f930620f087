#!/bin/bash
# Pseudo-header sums after the first pieces are issued in seg_live_varlen_kernel: the varlen pool tests,
# then the pool probe (live run-length x depth sweep) and the pool layouts' read floors in one session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r5y}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_varlen_pool.py \
  tests/test_gpu_parity.py > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
POOL_LIVE=1 timeout -k 10 400 python -u tools/varlen_pool_probe.py pool1520 pool2k pool1520mix pool2kmix > $O/${T}_varlen_pool_probe.jsonl \
  2> $O/${T}_varlen_pool_probe.err || { tail $O/${T}_varlen_pool_probe.err; exit 1; }
timeout -k 10 400 tools/build/live_read_probe seg1520 1520 34 1480 seg2k 2048 84 1480 seg1520mix 1520 34 mix seg2kmix 2048 84 mix \
  > $O/${T}_live_read_probe.jsonl 2> $O/${T}_live_read_probe.err || { tail $O/${T}_live_read_probe.err; exit 1; }
python3 - $O/${T}_live_read_probe.jsonl $O/${T}_varlen_pool_probe.jsonl <<'PY'
import json, sys
best = {}
for l in open(sys.argv[1]):
    d = json.loads(l)
    k = d["layout"].replace("seg", "pool")
    if d["ms"] < best.get(k, (9,))[0]:
        best[k] = (d["ms"], d["form"], d["run"])
print("floors", best)
for l in open(sys.argv[2]):
    d = json.loads(l)
    print(d["layout"], d["form"], d["ms"], "frac_of_floor", round(best[d["layout"]][0] / d["ms"], 4), d["kernel"][:70])
PY
echo "session $T done"
