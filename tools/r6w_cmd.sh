#!/bin/bash
# Round 6, session W: the chain row's fragment read floor (live_read_probe frag2k) beside chain pass 1's
# run lengths in the one-record live stream (interleaved), then the default's kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6w}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 tools/build/live_read_probe frag2k 2048 42 1480 > $O/${T}_live_read_probe.jsonl 2> $O/${T}_live_read_probe.err \
  || { tail $O/${T}_live_read_probe.err; exit 1; }
for c in ${CONFIGS:-chains.s10 chains.s12 chains.s14 chains chains.s12.d4 chains.s10 chains.s12 chains.s14 chains chains.s12.d4 chains.k4}; do
  echo "== $c" >> $O/${T}_runs.log
  timeout -k 10 120 python tools/run_config.py $c 60 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
done
timeout -k 10 300 tools/build/live_read_probe frag2k 2048 42 1480 >> $O/${T}_live_read_probe.jsonl 2>> $O/${T}_live_read_probe.err \
  || { tail $O/${T}_live_read_probe.err; exit 1; }
grep "==\|ms=" $O/${T}_runs.log | cut -c1-200
python3 - $O/${T}_live_read_probe.jsonl <<'PY'
import json, sys
best = {}
for l in open(sys.argv[1]):
    d = json.loads(l)
    k = (d["layout"], d["form"])
    best.setdefault(k, []).append(d["ms"])
for k, v in sorted(best.items()):
    print("floor", k, min(v), "x0.703125 =", round(min(v) * 0.703125, 4))
PY
echo "session $T done"
