#!/bin/bash
# Part B: per-row PMC of the packet-stream rows, the C driver's burst latency tables, the NIC-ring
# probe and the instruction mix of the sparse layouts, on the same sources.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r4zk}
O=gpurun_out
bash tools/gpu_pmc_all.sh $T rx rx6 rxmix rxb txb tx tx_nb rx_nb tx_nb2k rx_nb2k rx_nb2kv tx_nb2kv rx_ring tx_ring rx_ringv tx_ringv || exit 1
timeout -k 10 300 tools/build/burst_latency > $O/${T}_burst_latency.jsonl 2> $O/${T}_burst_latency.err || { tail $O/${T}_burst_latency.err; exit 1; }
timeout -k 10 120 tools/build/burst_latency zc > $O/${T}_burst_zc.jsonl 2> $O/${T}_burst_zc.err || { tail $O/${T}_burst_zc.err; exit 1; }
timeout -k 10 500 python -u tools/ring_probe.py > $O/${T}_ring_probe.jsonl 2> $O/${T}_ring_probe.err || { tail $O/${T}_ring_probe.err; exit 1; }
for c in rx_nb2k rx_ring rx_nb2kv; do bash tools/gpu_instmix.sh $T $c > /dev/null || exit 1; done
python3 tools/instmix_summary.py $O/${T}_*_instmix > $O/${T}_instmix.txt || exit 1
echo "session $T done"
