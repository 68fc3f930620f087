# Tx write-back call: packet-batch GPU tests, then the write-back sweep. Usage: bash ... <tag>
set -o pipefail
T=${1:-r1tx}
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_packets.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/tx_sweep.py > gpurun_out/${T}_sweep.jsonl 2> gpurun_out/${T}_sweep.err || exit $?
cat gpurun_out/${T}_sweep.jsonl
