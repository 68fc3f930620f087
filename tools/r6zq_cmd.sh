#!/bin/bash
# Round 6, session ZQ: dense strided segment batches at lengths other than 1500 B — run lengths
# (NETCSUM_TUNE_TILE) for the lengths that fall below C2's rate at the default 16-segment runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
T=${1:-r6zq}
O=$R/gpurun_out; mkdir -p $O
run() { SLP_LENS=$1 SLP_RUNS=$2 timeout -k 10 200 python tools/seglen_probe.py >> $O/${T}_seglen.jsonl 2>> $O/${T}.err || { tail $O/${T}.err; exit 1; }; }
run 1024 -1,12,15,17,20,23,24,25,31
run 2048 -1,8,9,11,12,13,15
run 4096 -1,3,4,5,6,7
run 8192 -1,2,3,4,5
run 9000 -1,2,3,4,5
run 1500 -1,15,17
python3 - $O/${T}_seglen.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["len"], d["run"], d["ms"], d["frac_of_8TBps"], d["kernel"].split("segs_per_wave=")[-1])
PY
echo "session $T done"
