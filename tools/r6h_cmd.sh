#!/bin/bash
# Round 6, evidence A on the final sources: the -m gpu suite, smoke, the driver-shaped bench, C2 / C5
# kernel trace + PMC (bench.py matches the C5 summary by source hash at N > 1), the configs record, the
# one-GPU --gpus 2 rehearsal, and the C5 variant probe (ride-along: which box type this is).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6h}
O=gpurun_out; mkdir -p $O
bash tools/gpu_run.sh $T tests smoke bench prof profc5 configs || exit 1
NETCSUM_BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --segments 65536 --steps 50 \
    --warmup 10 > $O/${T}_dist2.json 2> $O/${T}_dist2.err || { tail -20 $O/${T}_dist2.err; exit 1; }
tail -1 $O/${T}_dist2.json | cut -c1-300
C5P_VARIANTS=kernel,run_probe,run_probe_sleep,nopseudo,d6,w4,w6,s8,s24,xcd0,touch0 timeout -k 10 400 python -u tools/c5_probe.py \
  > $O/${T}_c5_probe.jsonl 2> $O/${T}_c5_probe.err || { tail $O/${T}_c5_probe.err; exit 1; }
cat $O/${T}_c5_probe.jsonl
echo "session $T done"
