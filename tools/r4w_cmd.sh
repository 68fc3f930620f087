#!/bin/bash
# Round-4: the chunk-level select for the parse's variable-offset transport-field dword
# (pkt_dword_at): packet / ring parity on the GPU, then the NIC-ring probe against r4k's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4w}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_pktstream.py tests/test_gpu_ring_layouts.py tests/test_gpu_packets.py tests/test_gpu_packets_v6.py \
    > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
timeout -k 10 500 python -u tools/ring_probe.py > "$O/ring_probe.jsonl" 2> "$O/ring_probe.err" || { tail "$O/ring_probe.err"; exit 1; }
echo "session done"
