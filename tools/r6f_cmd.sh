#!/bin/bash
# Round 6, session F (= E with the gathered result stores; gather0 = per-wave stores): the segment stream kernel
# (seg_stream_kernel PH 1): the segment parity suites (incl. full-size C2 / C5), the C5 / C2 variant
# probe, the driver-shaped bench (with the C5 point's read ceilings and live translation counters).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"
export TMPDIR=/tmp
T=${1:-r6e}
O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs_full.py tests/test_gpu_varlen_pool.py tests/test_gpu_chains.py -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
C5P_VARIANTS=kernel,gather0,nopseudo,run_probe timeout -k 10 300 python -u tools/c5_probe.py > $O/${T}_c5_probe.jsonl 2> $O/${T}_c5_probe.err \
  || { tail $O/${T}_c5_probe.err; exit 1; }
cat $O/${T}_c5_probe.jsonl
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail $O/${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/${T}_bench.json'))
print(d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['roofline']['frac_of_run_stream_read_probe'])
print(json.dumps(d['c5_shard_point'])[:2500])"
for c in chains chains.x0 chains chains.x0; do
  timeout -k 10 120 python tools/run_config.py $c 40 > $O/${T}_run_$c.log 2>&1 || { tail $O/${T}_run_$c.log; exit 1; }
  echo "$c $(tail -1 $O/${T}_run_$c.log)"
done
echo "session $T done"
