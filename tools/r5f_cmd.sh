#!/bin/bash
# Round 5, session f: offset/length packet batches with the deferred pass — the NIC-ring probe's
# offset/length variants under rocprofv3 --kernel-trace --stats (stream kernel vs deferred pass), then
# the varlen pool tests and probes (session e's second half).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5f}
O=$PWD/gpurun_out; mkdir -p $O
RING_VARIANTS=offlen timeout -k 10 300 python -u tools/ring_probe.py > $O/${T}_ring_probe_offlen.jsonl 2> $O/${T}_ring_probe_offlen.err \
  || { tail $O/${T}_ring_probe_offlen.err; exit 1; }
python3 - $O/${T}_ring_probe_offlen.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f"{d['layout']:9s} {d['form']:12s} {d['op']} {d['ms']:.4f}")
PY
( cd /tmp && RING_VARIANTS=offlen RING_N=1048576 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_offlen_trace -o offlen \
    --output-format csv -- python3 $OLDPWD/tools/ring_probe.py template ring > $O/${T}_offlen_trace.log 2>&1 ) \
  || { tail $O/${T}_offlen_trace.log; exit 1; }
f=$(ls $O/${T}_offlen_trace/*/offlen_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && cut -c1-160 "$f" | head -12
echo "session $T done"
