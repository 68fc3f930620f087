#!/bin/bash
# Round-4: the resident burst server — zero-copy host tests (modes 1-3), the idle stop / relaunch
# test, then the burst breakdown (tools/burst_latency.c zc) and the full burst table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4l}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_host.py \
    -k "zero_copy or burst_server" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 120 tools/build/burst_latency zc > "$O/burst_zc.jsonl" 2> "$O/burst_zc.err" || { tail -20 "$O/burst_zc.err"; exit 1; }
cat "$O/burst_zc.jsonl"
timeout -k 10 300 tools/build/burst_latency > "$O/burst_latency.jsonl" 2> "$O/burst_latency.err" || { tail -20 "$O/burst_latency.err"; exit 1; }
cat "$O/burst_latency.jsonl"
