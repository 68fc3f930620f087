#!/bin/bash
# Round 6, session B: the advisor fixes' and plan-identity GPU tests, the first-batch probe, the driver-shaped bench (c5_shard_point with its
# read ceilings), the one-GPU two-rank rehearsal (the per-rank fields), then session A's C5 probes
# and translation / L2 counters (tools/r6a_cmd.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6b}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_plans.py tests/test_gpu_ring_layouts.py tests/test_gpu_burst_server.py \
  tests/test_gpu_varlen_pool.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "deferred or burst or pool or plan" \
  > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
timeout -k 10 300 python -u tools/plan_ahead_probe.py > $O/${T}_plan_ahead_probe.jsonl 2> $O/${T}_plan_ahead_probe.err \
  || { tail $O/${T}_plan_ahead_probe.err; exit 1; }
cat $O/${T}_plan_ahead_probe.jsonl
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail $O/${T}_bench.err; exit 1; }
cat $O/${T}_bench.json
NETCSUM_BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --segments 65536 --steps 50 \
    --warmup 10 > $O/${T}_dist2.json 2> $O/${T}_dist2.err || { tail -20 $O/${T}_dist2.err; exit 1; }
cat $O/${T}_dist2.json
bash tools/r6a_cmd.sh ${T}a
