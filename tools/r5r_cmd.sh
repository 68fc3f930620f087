#!/bin/bash
# Live-sector read floors of the varlen pool layouts, uniform and mixed segment lengths
# (tools/live_read_probe.hip, LEN `mix`), beside the product's plans on the same layouts
# (tools/varlen_pool_probe.py) in the same session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r5r}
O=gpurun_out; mkdir -p $O
timeout -k 10 300 tools/build/live_read_probe seg1520 1520 34 1480 seg2k 2048 84 1480 seg1520mix 1520 34 mix seg2kmix 2048 84 mix \
  > $O/${T}_live_read_probe.jsonl 2> $O/${T}_live_read_probe.err || { tail $O/${T}_live_read_probe.err; exit 1; }
timeout -k 10 300 python -u tools/varlen_pool_probe.py pool1520 pool2k pool1520mix pool2kmix > $O/${T}_varlen_pool_probe.jsonl \
  2> $O/${T}_varlen_pool_probe.err || { tail $O/${T}_varlen_pool_probe.err; exit 1; }
python3 - $O/${T}_live_read_probe.jsonl $O/${T}_varlen_pool_probe.jsonl <<'PY'
import json, sys
best = {}
for l in open(sys.argv[1]):
    d = json.loads(l)
    k = d["layout"].replace("seg", "pool")
    best[k] = min(best.get(k, 9), d["ms"])
    print(d["layout"], d["form"], d["run"], d["pass"], d["ms"], d["frac_of_8TBps"])
for l in open(sys.argv[2]):
    d = json.loads(l)
    if d["form"] == "default":
        print("plan", d["layout"], d["ms"], "floor", best.get(d["layout"]), "frac_of_floor", round(best.get(d["layout"], 0) / d["ms"], 4), d["kernel"][:60])
PY
echo "session $T done"
