set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_host.py tests/test_gpu_pktstream.py tests/test_gpu_packets.py tests/test_gpu_packets_v6.py tests/test_gpu_offload.py tests/test_gpu_threads.py -m gpu > $O/r3m_tests.log 2>&1 || { tail -30 $O/r3m_tests.log; exit 1; }
tail -2 $O/r3m_tests.log
timeout -k 10 500 python -u tools/pkt_stream_sweep.py > $O/r3m_pkt_sweep.jsonl 2>&1 || { tail -5 $O/r3m_pkt_sweep.jsonl; exit 1; }
python3 -c "
import json
rows=[json.loads(l) for l in open('$O/r3m_pkt_sweep.jsonl') if l.startswith('{')]
for r in rows: print({k:v for k,v in r.items() if k not in ('kernel_rx','kernel_tx')})
"
