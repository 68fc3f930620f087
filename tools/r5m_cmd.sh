#!/bin/bash
# Round-5 evidence on the final sources, part A: the whole -m gpu suite, smoke, the driver-shaped
# bench, rocprofv3 kernel trace + PMC of C2 and of the C5 shard (the summary bench.py matches by source
# hash at N > 1), the configs record, and the one-GPU rehearsal of `bench.py --gpus 2`.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r5m}
O=gpurun_out
bash tools/gpu_run.sh $T tests smoke bench prof profc5 configs || exit 1
NETCSUM_BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --segments 65536 --steps 50 \
    --warmup 10 > $O/${T}_dist2.json 2> $O/${T}_dist2.err || { tail -20 $O/${T}_dist2.err; exit 1; }
cat $O/${T}_dist2.json
echo "session $T done"
