#!/bin/bash
# Round 5, session e: ring plans (ring-layout tests + the NIC-ring probe), the a3/a4 varlen batch on
# pool-buffer layouts (tools/varlen_pool_probe.py), and the live-sector read floors of the segment and
# chain-fragment layouts (tools/live_read_probe.hip).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5e}
O=gpurun_out; mkdir -p $O
SKIP_TESTS=${SKIP_TESTS:-} bash tools/r5b_cmd.sh $T || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_varlen_pool.py tests/test_gpu_parity.py > $O/${T}_varlen_tests.log 2>&1 || { tail -40 $O/${T}_varlen_tests.log; exit 1; }
tail -2 $O/${T}_varlen_tests.log
L=$PWD/uc-tcp-ip_amd
for lib in libnetcsum_mi355x.so build/libnetcsum_vlB.so build/libnetcsum_r4base.so; do
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
