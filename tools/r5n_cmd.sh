#!/bin/bash
# Round-5 evidence on the final sources, part B: per-row PMC sessions (tools/gpu_pmc_all.sh), the C
# driver's burst latency table and breakdown, and the NIC-ring probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5n}
O=gpurun_out
bash tools/gpu_pmc_all.sh $T || exit 1
timeout -k 10 300 tools/build/burst_latency > $O/${T}_burst_latency.jsonl 2> $O/${T}_burst_latency.err || { tail $O/${T}_burst_latency.err; exit 1; }
timeout -k 10 120 tools/build/burst_latency zc > $O/${T}_burst_zc.jsonl 2> $O/${T}_burst_zc.err || { tail $O/${T}_burst_zc.err; exit 1; }
timeout -k 10 500 python -u tools/ring_probe.py > $O/${T}_ring_probe.jsonl 2> $O/${T}_ring_probe.err || { tail $O/${T}_ring_probe.err; exit 1; }
echo "session $T done"
