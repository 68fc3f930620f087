#!/bin/bash
# Pipe-kernel experiment builds (tools/build_pipe_exp.sh: NETCSUM_PIPE_EXP 1 = first chunk row plain,
# 2 = plain touch of the segment two ahead) against the product on the varlen pool layouts, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r5q}
O=gpurun_out; mkdir -p $O
L=$PWD/uc-tcp-ip_amd
for r in 1 2; do
for lib in libnetcsum_mi355x.so build/libnetcsum_pipe1.so build/libnetcsum_pipe2.so; do
  tag=$(basename $lib .so)
  NETCSUM_LIB=$L/$lib timeout -k 10 300 python -u tools/varlen_pool_probe.py pool1520 pool2k pool1520mix pool2kmix > $O/${T}_${tag}_$r.jsonl 2> $O/${T}_$tag.err \
    || { tail $O/${T}_$tag.err; exit 1; }
  python3 - $O/${T}_${tag}_$r.jsonl $tag <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f"{sys.argv[2][12:]:8s} {d['layout']:12s} {d['form']:8s} {d['ms']:.4f} {d['frac_of_8TBps']:.3f} {d.get('parity_sample_ok', '')} {d['kernel'][:60]}")
PY
done
done
echo "session $T done"
