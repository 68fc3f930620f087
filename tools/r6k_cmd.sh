#!/bin/bash
# Round 6, session K: chain pass 1 compiled for 5 waves per SIMD (chains.w5) against the default, and the
# C5 shard's placement diagnostics (a second allocation of the same shard; pseudo-headers and results
# inside the segments' allocation) beside the kernel and its probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6k}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chains.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
for c in; do
  timeout -k 10 120 python tools/run_config.py $c 40 >> $O/${T}_chains_runs.log 2>&1 || { tail $O/${T}_chains_runs.log; exit 1; }
done
grep "ms=" $O/${T}_chains_runs.log
C5P_VARIANTS=kernel,run_probe,alloc2,alloc2_run_probe,onealloc,seg1_out2,seg2_out1,seg1_ph2_out2 timeout -k 10 400 python -u tools/c5_probe.py \
  > $O/${T}_c5_probe.jsonl 2> $O/${T}_c5_probe.err || { tail $O/${T}_c5_probe.err; exit 1; }
cut -c1-200 $O/${T}_c5_probe.jsonl
echo "session $T done"
