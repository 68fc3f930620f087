#!/bin/bash
# Round 6, evidence A on the final sources (after the chain row's one-record live pass 1): the -m gpu
# suite, smoke, the driver-shaped bench, C2 / C5 kernel trace + PMC, the configs record, the one-GPU
# --gpus 2 rehearsal, and the chain row's fragment read floor interleaved with the chain batch (default
# and the tiled pass 1) on the same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6z}
O=gpurun_out; mkdir -p $O
bash tools/gpu_run.sh $T tests smoke bench prof profc5 configs || exit 1
NETCSUM_BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --segments 65536 --steps 50 \
    --warmup 10 > $O/${T}_dist2.json 2> $O/${T}_dist2.err || { tail -20 $O/${T}_dist2.err; exit 1; }
tail -1 $O/${T}_dist2.json | cut -c1-300
timeout -k 10 300 tools/build/live_read_probe frag2k 2048 42 1480 > $O/${T}_live_read_probe.jsonl 2> $O/${T}_live_read_probe.err \
  || { tail $O/${T}_live_read_probe.err; exit 1; }
for c in chains chains.k4 chains chains.k4 chains; do
  echo "== $c" >> $O/${T}_chains_runs.log
  timeout -k 10 120 python tools/run_config.py $c 60 >> $O/${T}_chains_runs.log 2>&1 || { tail $O/${T}_chains_runs.log; exit 1; }
done
timeout -k 10 300 tools/build/live_read_probe frag2k 2048 42 1480 >> $O/${T}_live_read_probe.jsonl 2>> $O/${T}_live_read_probe.err \
  || { tail $O/${T}_live_read_probe.err; exit 1; }
grep "==\|ms=" $O/${T}_chains_runs.log | cut -c1-200
python3 - $O/${T}_live_read_probe.jsonl <<'PY'
import json, sys
best = {}
for l in open(sys.argv[1]):
    d = json.loads(l)
    best.setdefault((d["layout"], d["form"], d["run"]), []).append(d["ms"])
k, v = min(best.items(), key=lambda kv: min(kv[1]))
print("floor", k, min(v), "x 737280/2^20 =", round(min(v) * 0.703125, 4), "ms")
PY
echo "session $T done"
