# Packet + chain kernels call: their GPU tests, the Tx write-back sweep, secondary configs. Usage: bash ... <tag>
set -o pipefail
T=${1:-r1tc}
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_packets.py tests/test_gpu_chains.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/tx_sweep.py > gpurun_out/${T}_tx_sweep.jsonl 2> gpurun_out/${T}_tx_sweep.err || exit $?
cat gpurun_out/${T}_tx_sweep.jsonl
timeout -k 10 400 python -u tools/bench_configs.py > gpurun_out/${T}_configs.json 2> gpurun_out/${T}_configs.err || exit $?
cat gpurun_out/${T}_configs.json
