#!/bin/bash
# Round 6, session A: the C5 shard's per-GPU deficit (verdict r5 item 1). The C5 / C2 variant probe
# (tools/c5_probe.py), then the translation and L2 request counters of C2 and C5 (bench.py's launch,
# which also runs both read probes over the same bytes), one rocprofv3 --pmc pass per counter group.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6a}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u tools/c5_probe.py > $O/${T}_c5_probe.jsonl 2> $O/${T}_c5_probe.err || { tail $O/${T}_c5_probe.err; exit 1; }
cat $O/${T}_c5_probe.jsonl
A="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum"
B="TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum TCC_TAG_STALL_sum"
ARGS=""
for sz in 1048576 16777216; do
  for p in A B C; do
    eval "CN=\$$p"
    D=$O/${T}_pmc_${sz}_$p
    ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CN -d $D -o p --output-format csv \
        -- python3 $R/bench.py --steps 3 --warmup 1 --ramp-seconds 0 --no-cpu-baseline --no-c5-point --pmc off \
           --segments $sz > $D.json 2> $D.err ) || { tail -5 $D.err; exit 1; }
    ARGS="$ARGS n${sz}_$p=$D"
  done
done
python3 tools/pmc_generic.py $O/${T}_xlat_pmc.json $ARGS || exit 1
python3 - $O/${T}_xlat_pmc.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for lab, ks in d["passes"].items():
    for k, v in ks.items():
        print(lab, k[:60], {c: round(x) for c, x in v.items()})
PY
echo "session $T done"
