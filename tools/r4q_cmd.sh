#!/bin/bash
# Round-4: burst server with per-wave acquire and per-block release — host/thread GPU tests, burst
# breakdown and table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4q}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_host.py \
    tests/test_gpu_threads.py tests/test_gpu_offload.py > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 120 tools/build/burst_latency zc > "$O/burst_zc.jsonl" 2> "$O/burst_zc.err" || { tail -20 "$O/burst_zc.err"; exit 1; }
cat "$O/burst_zc.jsonl"
timeout -k 10 300 tools/build/burst_latency > "$O/burst_latency.jsonl" 2> "$O/burst_latency.err" || { tail -20 "$O/burst_latency.err"; exit 1; }
python3 -c "
import json,sys
for l in open('$O/burst_latency.jsonl'):
    d=json.loads(l); print({k:v for k,v in d.items() if k in ('frames','rx_host_us_auto','tx_host_us_auto','rx_host_us_server','tx_host_us_server','all_delivered_auto')})
"
