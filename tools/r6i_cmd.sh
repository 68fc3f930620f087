#!/bin/bash
# Round 6, evidence B on the final sources: every DESIGN §9 row's kernel trace + FETCH_SIZE / WRITE_SIZE
# PMC (tools/gpu_pmc_all.sh; the Tx rows also their L2 write requests), keyed by kernel-source hash.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r6i}
bash tools/gpu_pmc_all.sh $T || exit 1
echo "session $T done"
