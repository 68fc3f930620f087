set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pktstream.py tests/test_gpu_chains.py tests/test_gpu_hdrstream.py tests/test_gpu_packets.py tests/test_gpu_packets_v6.py -m gpu > $O/r3i_tests.log 2>&1 || { tail -30 $O/r3i_tests.log; exit 1; }
tail -2 $O/r3i_tests.log
timeout -k 10 300 python -u tools/pkt_gap_probe.py > $O/r3i_gap_probe.jsonl 2>&1 || { tail -5 $O/r3i_gap_probe.jsonl; exit 1; }
cat $O/r3i_gap_probe.jsonl
timeout -k 10 300 python -u bench.py > $O/r3i_bench.log 2>&1 || { tail -5 $O/r3i_bench.log; exit 1; }
tail -1 $O/r3i_bench.log
