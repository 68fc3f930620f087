#!/bin/bash
# Round-4 GPU command: driver-shaped bench (with the C5 retention point) and the --gpus 2 launcher
# rehearsal on one GPU (gloo, ranks folded onto the one device). Every GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4a}
mkdir -p "$O"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err" &&
NETCSUM_BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --segments 65536 --steps 50 \
    --warmup 10 > "$O/dist2.json" 2> "$O/dist2.err"
rc=$?
tail -c 600 "$O/bench.json"; echo; cat "$O/dist2.json"; tail -5 "$O/dist2.err"
exit $rc
