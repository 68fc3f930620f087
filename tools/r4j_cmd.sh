#!/bin/bash
# Round-4 evidence on the final sources, part A: the whole -m gpu suite, smoke, the driver-shaped
# bench, rocprofv3 kernel trace + PMC of C2 and of the C5 shard, the configs record.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r4j}
bash tools/gpu_run.sh $T tests smoke bench prof profc5 configs
