set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python tools/rx_order_probe.py > gpurun_out/r1t_rx_order.jsonl 2> gpurun_out/r1t_rx_order.err || exit $?
cat gpurun_out/r1t_rx_order.jsonl
