#!/bin/bash
# Round-4 session: the whole -m gpu suite and smoke, the driver-shaped bench, the ring probe and the
# zero-copy burst breakdown. Each GPU step under its own limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4e}
mkdir -p "$O"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['frac'],d['roofline']['traffic_over_algorithmic'],d.get('c5_shard_point',{}).get('value_per_gpu'),d['c1_per_datagram'].get('gpu_dropin_us_per_call'))"
timeout -k 10 500 python -u tools/ring_probe.py > "$O/ring_probe.jsonl" 2> "$O/ring_probe.err" || { tail -20 "$O/ring_probe.err"; exit 1; }
python3 - "$O/ring_probe.jsonl" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d["layout"], d["form"], d["op"], d["ms"], d["frac_of_8TBps"], d["Mframes_per_s"], d.get("all_valid"), d.get("bytes_equal_first_tx"))
PY
timeout -k 10 120 tools/build/burst_latency zc > "$O/burst_zc.jsonl" 2> "$O/burst_zc.err" || { tail -20 "$O/burst_zc.err"; exit 1; }
cat "$O/burst_zc.jsonl"
