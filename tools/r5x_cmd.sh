#!/bin/bash
# Round-5 evidence on the final sources, part B: per-row PMC sessions (tools/gpu_pmc_all.sh, the pool
# layouts included), the C driver's burst latency table and breakdown, the NIC-ring probe, the pool
# probe and the live-sector read floors of the pool and fragment layouts (runs of 8 / 16 / 32).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5x}
O=gpurun_out
mkdir -p $O
bash tools/gpu_pmc_all.sh $T || exit 1
timeout -k 10 300 tools/build/burst_latency > $O/${T}_burst_latency.jsonl 2> $O/${T}_burst_latency.err || { tail $O/${T}_burst_latency.err; exit 1; }
timeout -k 10 120 tools/build/burst_latency zc > $O/${T}_burst_zc.jsonl 2> $O/${T}_burst_zc.err || { tail $O/${T}_burst_zc.err; exit 1; }
timeout -k 10 500 python -u tools/ring_probe.py > $O/${T}_ring_probe.jsonl 2> $O/${T}_ring_probe.err || { tail $O/${T}_ring_probe.err; exit 1; }
timeout -k 10 300 python -u tools/varlen_pool_probe.py > $O/${T}_varlen_pool_probe.jsonl 2> $O/${T}_varlen_pool_probe.err || { tail $O/${T}_varlen_pool_probe.err; exit 1; }
timeout -k 10 400 tools/build/live_read_probe seg1520 1520 34 1480 seg2k 2048 84 1480 seg1520mix 1520 34 mix seg2kmix 2048 84 mix \
  frag2k 2048 42 1480 > $O/${T}_live_read_probe.jsonl 2> $O/${T}_live_read_probe.err || { tail $O/${T}_live_read_probe.err; exit 1; }
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
    if d["form"] == "default" and d["layout"] in best:
        print("plan", d["layout"], d["ms"], "floor", best[d["layout"]], "frac_of_floor", round(best[d["layout"]][0] / d["ms"], 4), d["kernel"][:70])
PY
echo "session $T done"
