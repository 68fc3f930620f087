#!/bin/bash
# Round-4 session b: bounded packet stream + zero-copy host bursts — parity (new ring tests, the
# packet and host suites), then the ring probe (every layout x bound x form) and the C driver's
# burst latency. Each GPU step under its own limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4b}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_ring_layouts.py \
    tests/test_gpu_host.py tests/test_gpu_pktstream.py tests/test_gpu_packets.py tests/test_gpu_packets_v6.py \
    tests/test_gpu_offload.py tests/test_gpu_threads.py > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
# (full burst-size table: tools/build/burst_latency without "zc")

timeout -k 10 120 tools/build/burst_latency zc > "$O/burst_zc.jsonl" 2> "$O/burst_zc.err" || { tail -20 "$O/burst_zc.err"; exit 1; }
cat "$O/burst_zc.jsonl"
timeout -k 10 500 python -u tools/ring_probe.py > "$O/ring_probe.jsonl" 2> "$O/ring_probe.err" || { tail -20 "$O/ring_probe.err"; exit 1; }
python3 - "$O/ring_probe.jsonl" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d["layout"], d["form"], d["op"], d["ms"], d["frac_of_8TBps"], d["Mframes_per_s"], d.get("all_valid"), d.get("bytes_equal_first_tx"))
PY
