#!/bin/bash
# Round-4 evidence after the in-window datagram change (netcsum_pktstream.hip), part A: the whole
# -m gpu suite, smoke, the driver-shaped bench and the configs record. (The headline stream
# kernel's sources are unchanged: its rocprof / PMC evidence stays r4j's.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_run.sh ${1:-r4z} tests smoke bench configs || exit 1
echo "session done"
