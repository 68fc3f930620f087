#!/bin/bash
# Round 6, session ZR: dense strided runs chosen by bytes (runs of 16 unless 16 segments' bytes are a
# multiple of 16 KiB or past 48 KiB): the -m gpu suite, then the segment-length probe at the default
# launch (C2's 1500 B keeps runs of 16), then the driver-shaped bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
T=${1:-r6zr}
O=$R/gpurun_out; mkdir -p $O
bash tools/gpu_run.sh $T tests || exit 1
timeout -k 10 300 python tools/seglen_probe.py > $O/${T}_seglen.jsonl 2> $O/${T}.err || { tail $O/${T}.err; exit 1; }
python3 - $O/${T}_seglen.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["len"], d["ms"], d["frac_of_8TBps"], d["kernel"].split("segs_per_wave=")[-1])
PY
bash tools/gpu_run.sh $T bench || exit 1
echo "session $T done"
