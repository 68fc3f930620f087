#!/bin/bash
# Round-5 evidence after the last changes to csrc/netcsum_stream.hip and netcsum_chains.hip: the
# -m gpu suite, smoke, the driver-shaped bench, C2 / C5 kernel trace + PMC (bench.py matches the C5
# summary by source hash at N > 1), the configs record, the one-GPU --gpus 2 rehearsal, the PMC rows
# of the kernels in those files (C4, the pool layouts, chains), the pool probe and the pool read floors.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5aa}
O=gpurun_out; mkdir -p $O
bash tools/gpu_run.sh $T tests smoke bench prof profc5 configs || exit 1
NETCSUM_BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --segments 65536 --steps 50 \
    --warmup 10 > $O/${T}_dist2.json 2> $O/${T}_dist2.err || { tail -20 $O/${T}_dist2.err; exit 1; }
bash tools/gpu_pmc_all.sh $T c4 pool1520 pool1520mix pool2k pool2kmix chains || exit 1
timeout -k 10 300 python -u tools/varlen_pool_probe.py > $O/${T}_varlen_pool_probe.jsonl 2> $O/${T}_varlen_pool_probe.err || { tail $O/${T}_varlen_pool_probe.err; exit 1; }
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
    if d["form"] == "default" and d["layout"] in best:
        print("plan", d["layout"], d["ms"], "floor", best[d["layout"]], "frac_of_floor", round(best[d["layout"]][0] / d["ms"], 4), d["kernel"][:70])
    elif d["form"] == "default":
        print("plan", d["layout"], d["ms"], d["kernel"][:70])
PY
echo "session $T done"
