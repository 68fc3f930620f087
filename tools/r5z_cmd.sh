#!/bin/bash
# The varlen sampler with its loads batched (varlen_runlen_kernel / the live kernel's sampler block):
# the varlen GPU tests, then C4 and a pool layout by events and under a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-r5z}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_varlen_pool.py \
  tests/test_gpu_parity.py > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
for c in c4 pool1520mix c4 pool1520mix; do
  timeout -k 10 120 python -u tools/run_config.py $c 200 >> $O/${T}_runs.log 2>&1 || { tail $O/${T}_runs.log; exit 1; }
done
grep -v amdgpu.ids $O/${T}_runs.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${T}_trace -o trace -- python3 tools/run_config.py c4 30 > /dev/null 2> $O/${T}_trace.err \
  || { tail $O/${T}_trace.err; exit 1; }
f=$(ls $O/${T}_trace/*/trace_kernel_stats.csv $O/${T}_trace/trace_kernel_stats.csv 2>/dev/null | head -1)
grep -i "runlen\|varlen" $f | cut -c1-200
echo "session $T done"
