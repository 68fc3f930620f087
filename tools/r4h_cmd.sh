#!/bin/bash
# Round-4: dynamic instruction mix (SQ counters, one rocprofv3 --pmc pass each) of the packet stream's
# read forms on three layouts (tools/gpu_instmix.sh), summarised by tools/instmix_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for c in rx.b0 rx rx_nb2k.b0 rx_nb2k rx_nb2k.b1 rx_ring.b0 rx_ring rx_ring.b2.s32; do
  bash tools/gpu_instmix.sh r4h $c || exit 1
done
python3 tools/instmix_summary.py gpurun_out/r4h_*_instmix | tee gpurun_out/r4h_instmix.txt
