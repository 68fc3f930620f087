#!/bin/bash
# Round 5, session k: the whole -m gpu suite, the varlen pool probe with the pipe geometries, and on
# the same box the chain row's fragments (tools/frag_stream_probe.py) beside their live-sector floor.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5k}
O=$PWD/gpurun_out; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PYT -m gpu tests > $O/${T}_gpu_tests.log 2>&1 || { tail -40 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
POOL_PIPES=1 timeout -k 10 400 python -u tools/varlen_pool_probe.py pool1520 pool2k pool1520mix > $O/${T}_varlen_pool_probe.jsonl \
  2> $O/${T}_varlen_pool_probe.err || { tail $O/${T}_varlen_pool_probe.err; exit 1; }
python3 - $O/${T}_varlen_pool_probe.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f"{d['layout']:12s} {d['form']:12s} {d['ms']:.4f} {d['frac_of_8TBps']:.3f} {d.get('parity_sample_ok', '')} {d['kernel'][:90]}")
PY
timeout -k 10 300 tools/build/live_read_probe seg1520 1520 34 1480 seg2k 2048 84 1480 frag2k 2048 42 1480 \
  > $O/${T}_live_read_probe.jsonl 2> $O/${T}_live_read_probe.err || { tail $O/${T}_live_read_probe.err; exit 1; }
python3 - $O/${T}_live_read_probe.jsonl <<'PY'
import json, sys
best = {}
for l in open(sys.argv[1]):
    d = json.loads(l)
    k = d['layout']
    if k not in best or d['ms'] < best[k]['ms']:
        best[k] = d
for k, d in best.items():
    print(f"floor {k:8s} {d['form']:14s} R{d['run']:<3d} {d['ms']:.4f} {d['frac_of_8TBps']:.4f}")
PY
timeout -k 10 300 python -u tools/frag_stream_probe.py > $O/${T}_frag_stream_probe.jsonl 2> $O/${T}_frag_stream_probe.err \
  || { tail $O/${T}_frag_stream_probe.err; exit 1; }
python3 - $O/${T}_frag_stream_probe.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d['pass'], d['pitch'], {k: v for k, v in d.items() if k.endswith('_ms')})
PY
echo "session $T done"
