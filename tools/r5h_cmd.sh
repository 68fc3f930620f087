#!/bin/bash
# Round 5, session h: offset/length ring plans + deferred pass (tests, NIC-ring probe, kernel trace),
# then the a3/a4 varlen pool layouts (tests, probe vs the round-4 library) and the live-sector floors.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5h}
O=$PWD/gpurun_out; mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PYT tests/test_gpu_ring_layouts.py tests/test_gpu_varlen_pool.py > $O/${T}_tests.log 2>&1 \
  || { tail -40 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
RING_VARIANTS=${RING_VARIANTS:-} timeout -k 10 400 python -u tools/ring_probe.py > $O/${T}_ring_probe.jsonl 2> $O/${T}_ring_probe.err \
  || { tail $O/${T}_ring_probe.err; exit 1; }
python3 - $O/${T}_ring_probe.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    if d['form'] in ('strided.plan', 'strided.b0', 'strided.b2', 'offlen', 'offlen.lanegroup'):
        print(f"{d['layout']:9s} {d['form']:16s} {d['op']} {d['ms']:.4f} {d.get('plan', '')} {d['kernel'][-40:]}")
PY
L=$PWD/uc-tcp-ip_amd
for lib in libnetcsum_mi355x.so build/libnetcsum_r4base.so; do
  tag=$(basename $lib .so)
  NETCSUM_LIB=$L/$lib timeout -k 10 400 python -u tools/varlen_pool_probe.py > $O/${T}_varlen_pool_probe_$tag.jsonl 2> $O/${T}_varlen_pool_probe_$tag.err \
    || { tail $O/${T}_varlen_pool_probe_$tag.err; exit 1; }
  python3 - $O/${T}_varlen_pool_probe_$tag.jsonl $tag <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f"{sys.argv[2][12:]:8s} {d['layout']:12s} {d['form']:8s} {d['ms']:.4f} {d['frac_of_8TBps']:.3f} {d.get('parity_sample_ok', '')} {d['kernel'][:60]}")
PY
done
timeout -k 10 400 tools/build/live_read_probe seg1520 1520 34 1480 seg2k 2048 84 1480 frag2k 2048 42 1480 \
  > $O/${T}_live_read_probe.jsonl 2> $O/${T}_live_read_probe.err || { tail $O/${T}_live_read_probe.err; exit 1; }
python3 - $O/${T}_live_read_probe.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    if d['pass'] == 1:
        print(f"{d['layout']:8s} {d['form']:14s} R{d['run']:<3d} {d['ms']:.4f} {d['frac_of_8TBps']:.4f}")
PY
echo "session $T done"
