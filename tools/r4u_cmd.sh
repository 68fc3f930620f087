#!/bin/bash
# Round-4: why the C5 shard (16 M x 1500 B, 25.4 GB per GPU) runs further below its run-stream read
# probe than C2 does on some boxes (r4j: 3.78 ms against a 3.45-ms probe; C2: 99 % of its probe) —
# the default against no pseudo-headers, the plain block order, no row touch, 4 / 6 waves per SIMD
# and runs of 32, each with the read probe over the same bytes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4u}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_host.py \
    -k "burst_server or zero_copy" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
i=0
for v in "" "--pseudo-len 0" "--tune xcd=0" "--tune touch=0" "--tune waves=4" "--tune waves=6" "--tune tile=32" ""; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --segments 16777216 --steps 30 --warmup 5 --no-cpu-baseline --pmc off \
      --no-c5-point $v > "$O/c5_$i.json" 2> "$O/c5_$i.err" || { tail -5 "$O/c5_$i.err"; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$O/c5_$i.json')); r=d['roofline']
print('$v', d['value'], r['kernel_ms'], r['run_stream_read_probe_GBps'], r['frac_of_run_stream_read_probe'], r['frac'])"
done
