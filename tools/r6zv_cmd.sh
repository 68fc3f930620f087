#!/bin/bash
# Round 6, session ZV: dense IPv4 / IPv6 runs of long datagrams chosen by bytes (runs of 8 unless their
# bytes are a multiple of 16 KiB or past 48 KiB, then about 10 KiB): the -m gpu suite, the packet-length
# probe at the default launch, the driver-shaped bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
T=${1:-r6zv}
O=$R/gpurun_out; mkdir -p $O
bash tools/gpu_run.sh $T tests || exit 1
PLP_KINDS=rx PLP_LENS=1500,2048,3000,4096,6000,8192,9000 timeout -k 10 300 python tools/pktlen_probe.py > $O/${T}_pktlen.jsonl 2> $O/${T}.err \
  || { tail $O/${T}.err; exit 1; }
python3 - $O/${T}_pktlen.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["len"], d["ms"], d["frac_of_8TBps"], d["kernel"].split("pkts_per_wave=")[-1])
PY
bash tools/gpu_run.sh $T bench || exit 1
echo "session $T done"
