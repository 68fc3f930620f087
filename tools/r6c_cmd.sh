#!/bin/bash
# Round 6, session C: the compacted live-sector stream of pool segments (seg_live_varlen_kernel CMP):
# its parity tests, the pool probe (default = compacted, "pieces" = round 5's live pieces), the read
# floors of the pool layouts and of the mixed NIC ring with the compacted forms, the ring probe's plan
# variants, and the first-batch probe with a planned id per layout.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6c}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_varlen_pool.py tests/test_gpu_plans.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
timeout -k 10 300 python -u tools/varlen_pool_probe.py pool1520mix pool2kmix pool1520 pool2k > $O/${T}_varlen_pool_probe.jsonl \
  2> $O/${T}_varlen_pool_probe.err || { tail $O/${T}_varlen_pool_probe.err; exit 1; }
cut -c1-400 $O/${T}_varlen_pool_probe.jsonl
timeout -k 10 500 tools/build/live_read_probe seg1520mix 1520 34 mix seg1520mixwin 1520 34 mixwin seg2kmixwin 2048 84 mixwin \
  seg1520 1520 34 1480 seg2k 2048 84 1480 ring 1520 14 ringmix > $O/${T}_live_read_probe.jsonl 2> $O/${T}_live_read_probe.err \
  || { tail $O/${T}_live_read_probe.err; exit 1; }
python3 - $O/${T}_live_read_probe.jsonl <<'PY'
import json, sys
best = {}
for l in open(sys.argv[1]):
    d = json.loads(l)
    k = (d["layout"], d["form"].split(".")[0])
    if d["ms"] < best.get(k, (9,))[0]:
        best[k] = (d["ms"], d["form"], d["run"])
for k, v in sorted(best.items()):
    print("floor", k, v)
PY
RING_VARIANTS=plan timeout -k 10 300 python -u tools/ring_probe.py ring > $O/${T}_ring_probe.jsonl 2> $O/${T}_ring_probe.err \
  || { tail $O/${T}_ring_probe.err; exit 1; }
cut -c1-300 $O/${T}_ring_probe.jsonl
timeout -k 10 300 python -u tools/plan_ahead_probe.py > $O/${T}_plan_ahead_probe.jsonl 2> $O/${T}_plan_ahead_probe.err \
  || { tail $O/${T}_plan_ahead_probe.err; exit 1; }
cut -c1-200 $O/${T}_plan_ahead_probe.jsonl
echo "session $T done"
