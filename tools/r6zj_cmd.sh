#!/bin/bash
# Round 6, session ZJ: counters of the C2 segment stream against the packed Rx kernel on the same
# 1 M x 1500 B (and C2 in Rx's shape: runs of 8, full residency) — HBM read requests and their size,
# L2 tag stalls, L1 -> L2 read latency, instruction mix and wave occupancy — one rocprofv3 --pmc pass
# per counter group, each its own run (tools/run_config.py, 5 launches), summarised by pmc_generic.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
T=${1:-r6zj}
O=$R/gpurun_out; mkdir -p $O
P1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_TAG_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
P2="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS"
ARGS=()
for c in ${CONFIGS:-c2 rx c2.s8.w0}; do
  for p in 1 2; do
    eval "CNT=\$P$p"
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $CNT -d $O/${T}_${c}_p$p -o p --output-format csv \
      -- python3 $R/tools/run_config.py $c 5 > $O/${T}_${c}_p$p.log 2>&1 ) || { tail -5 $O/${T}_${c}_p$p.log; exit 1; }
    ARGS+=("${c}_p$p=$O/${T}_${c}_p$p")
  done
done
python3 tools/pmc_generic.py $O/${T}_pmc.json "${ARGS[@]}" || exit 1
python3 - $O/${T}_pmc.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for lab, ks in d["passes"].items():
    for k, v in ks.items():
        if "fill_kernel" in k or "tx" in k.split("<")[-1][:40] and "rx" not in k: continue
        print(lab, k.split("(")[0].split("::")[-1][:50], {c: round(x) for c, x in v.items()})
PY
echo "session $T done"
