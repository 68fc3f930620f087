#!/bin/bash
# Round-4: sentinel pop / table prefix masks / 63-KiB live reach, and the resident burst server —
# packet, host and thread GPU tests, the burst breakdown and table, the ring probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4m}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_host.py \
    tests/test_gpu_ring_layouts.py tests/test_gpu_pktstream.py tests/test_gpu_packets.py tests/test_gpu_packets_v6.py \
    tests/test_gpu_offload.py tests/test_gpu_threads.py > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 120 tools/build/burst_latency zc > "$O/burst_zc.jsonl" 2> "$O/burst_zc.err" || { tail -20 "$O/burst_zc.err"; exit 1; }
cat "$O/burst_zc.jsonl"
timeout -k 10 300 tools/build/burst_latency > "$O/burst_latency.jsonl" 2> "$O/burst_latency.err" || { tail -20 "$O/burst_latency.err"; exit 1; }
cat "$O/burst_latency.jsonl"
timeout -k 10 500 python -u tools/ring_probe.py > "$O/ring_probe.jsonl" 2> "$O/ring_probe.err" || { tail -20 "$O/ring_probe.err"; exit 1; }
python3 - "$O/ring_probe.jsonl" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d["layout"], d["form"], d["op"], d["ms"], d["frac_of_8TBps"], d["Mframes_per_s"], d.get("all_valid"), d.get("bytes_equal_first_tx"))
PY
