#!/bin/bash
# Round 5, session c: experiment builds of the device plan (not the product): 1 = a constant plan
# (no sampling), 2 = persistent waves (grid = blocks per CU x 256, runs round-robin) with sampling,
# 3 = both; against the product build, on the template / 2-KiB / mixed rings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5c}
O=gpurun_out; mkdir -p $O
run() {   # tag lib [env]
  local tag=$1 lib=$2; shift 2
  env NETCSUM_LIB=$lib RING_VARIANTS=plan "$@" timeout -k 10 300 python -u tools/ring_probe.py template ring nb2k \
    > $O/${T}_${tag}.jsonl 2> $O/${T}_${tag}.err || { tail $O/${T}_${tag}.err; exit 1; }
  python3 - $O/${T}_${tag}.jsonl $tag <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    if d['form'] in ('strided.plan', 'strided.b0', 'strided.b2.s8', 'strided.b2.s32'):
        print(f"{sys.argv[2]:8s} {d['layout']:9s} {d['form']:16s} {d['op']} {d['ms']:.4f} {d.get('plan', '')}")
PY
}
L=$PWD/uc-tcp-ip_amd
run prod $L/libnetcsum_mi355x.so
run exp1 $L/build/libnetcsum_exp1.so
run exp2 $L/build/libnetcsum_exp2.so
run exp2b8 $L/build/libnetcsum_exp2.so NETCSUM_PLAN_BPC=8
run exp3 $L/build/libnetcsum_exp3.so
echo "session $T done"
