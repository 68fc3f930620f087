#!/bin/bash
# Round-4: burst server without per-wave fences (system-scope ring loads and result stores), default
# bound 2 / 24-KB runs — packet/host/thread GPU tests, burst breakdown and table, ring probe, the
# live-sector read probe with touch / 8-deep variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4p}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_host.py \
    tests/test_gpu_ring_layouts.py tests/test_gpu_pktstream.py tests/test_gpu_packets.py tests/test_gpu_packets_v6.py \
    tests/test_gpu_offload.py tests/test_gpu_threads.py > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 120 tools/build/burst_latency zc > "$O/burst_zc.jsonl" 2> "$O/burst_zc.err" || { tail -20 "$O/burst_zc.err"; exit 1; }
cat "$O/burst_zc.jsonl"
timeout -k 10 300 tools/build/burst_latency > "$O/burst_latency.jsonl" 2> "$O/burst_latency.err" || { tail -20 "$O/burst_latency.err"; exit 1; }
python3 -c "
import json,sys
for l in open('$O/burst_latency.jsonl'):
    d=json.loads(l); print({k:v for k,v in d.items() if k in ('frames','rx_host_us_auto','tx_host_us_auto','rx_host_us_server','tx_host_us_server','all_delivered_auto')})
"
timeout -k 10 500 python -u tools/ring_probe.py > "$O/ring_probe.jsonl" 2> "$O/ring_probe.err" || { tail -20 "$O/ring_probe.err"; exit 1; }
python3 - "$O/ring_probe.jsonl" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d["layout"], d["form"], d["op"], d["ms"], d["frac_of_8TBps"], d["Mframes_per_s"], d.get("all_valid"), d.get("bytes_equal_first_tx"))
PY
timeout -k 10 400 tools/build/live_read_probe > "$O/live_read_probe.jsonl" 2> "$O/live_read_probe.err" || { tail -20 "$O/live_read_probe.err"; exit 1; }
python3 -c "
import json
for l in open('$O/live_read_probe.jsonl'):
    d=json.loads(l); print(d['layout'],d['form'],d['run'],d['pass'],d['ms'],d['frac_of_8TBps'],d['sector_GBps'])
"
