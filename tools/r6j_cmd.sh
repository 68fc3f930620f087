#!/bin/bash
# Round 6, evidence C on the final sources: the pool probe (compacted live sectors and round 5's live
# pieces), the read floors (pool segments, the chain row's fragments, the NIC rings incl. the mixed ring
# with its 96-B header window) and the mixed ring floor's PMC traffic, the ring probe's plans, the
# first-batch probe and the chain row's batch times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6j}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/varlen_pool_probe.py > $O/${T}_varlen_pool_probe.jsonl 2> $O/${T}_varlen_pool_probe.err \
  || { tail $O/${T}_varlen_pool_probe.err; exit 1; }
timeout -k 10 600 tools/build/live_read_probe seg1520mix 1520 34 mix seg1520mixwin 1520 34 mixwin seg2kmixwin 2048 84 mixwin \
  seg1520 1520 34 1480 seg2k 2048 84 1480 frag2k 2048 42 1480 ring 1520 14 ringmix template 1520 14 1500 nb2k 2048 64 1500 \
  > $O/${T}_live_read_probe.jsonl 2> $O/${T}_live_read_probe.err || { tail $O/${T}_live_read_probe.err; exit 1; }
for v in "live.win 32" "compact.win 16"; do
  set -- $v
  ( cd /tmp && LRP_FORM=$1 LRP_RUN=$2 LRP_WARM=3 LRP_PASSES=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/${T}_ringfloor_$1 \
      -o f --output-format csv -- $R/tools/build/live_read_probe ring 1520 14 ringmix > /dev/null 2> $O/${T}_ringfloor_$1.err ) \
    || { tail $O/${T}_ringfloor_$1.err; exit 1; }
done
python3 - $O $T <<'PY'
import csv, glob, json, statistics, sys
O, T = sys.argv[1], sys.argv[2]
res = {}
for form in ("live.win", "compact.win"):
    vals = []
    for f in glob.glob(f"{O}/{T}_ringfloor_{form}/**/f_counter_collection.csv", recursive=True):
        vals += [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "probe_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
    res[form] = {"launches": len(vals), "FETCH_SIZE_KB_median": statistics.median(vals) if vals else None,
                 "hbm_read_bytes_per_launch": statistics.median(vals) * 1024 * 2 if vals else None}
json.dump(res, open(f"{O}/{T}_ring_floor_pmc.json", "w"), indent=1)
print(res)
PY
RING_VARIANTS=plan timeout -k 10 300 python -u tools/ring_probe.py > $O/${T}_ring_probe.jsonl 2> $O/${T}_ring_probe.err \
  || { tail $O/${T}_ring_probe.err; exit 1; }
timeout -k 10 300 python -u tools/plan_ahead_probe.py > $O/${T}_plan_ahead_probe.jsonl 2> $O/${T}_plan_ahead_probe.err \
  || { tail $O/${T}_plan_ahead_probe.err; exit 1; }
for c in chains chains chains.x0 chains.x0; do
  timeout -k 10 120 python tools/run_config.py $c 40 >> $O/${T}_chains_runs.log 2>&1 || { tail $O/${T}_chains_runs.log; exit 1; }
done
tail -4 $O/${T}_chains_runs.log
python3 - $O/${T}_live_read_probe.jsonl $O/${T}_varlen_pool_probe.jsonl <<'PY'
import json, sys
best = {}
for l in open(sys.argv[1]):
    d = json.loads(l)
    k = (d["layout"], d["form"].split(".")[0])
    if d["ms"] < best.get(k, (9,))[0]:
        best[k] = (d["ms"], d["form"], d["run"])
for k, v in sorted(best.items()):
    print("floor", k, v)
for l in open(sys.argv[2]):
    d = json.loads(l)
    print("pool", d["layout"], d["form"], d["ms"], d["kernel"][:70])
PY
echo "session $T done"
