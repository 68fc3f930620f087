set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 500 python -u tools/pkt_stream_sweep.py > $O/r3l_pkt_sweep.jsonl 2>&1 || { tail -5 $O/r3l_pkt_sweep.jsonl; exit 1; }
python3 -c "
import json
rows=[json.loads(l) for l in open('$O/r3l_pkt_sweep.jsonl') if l.startswith('{')]
for r in rows: print({k:v for k,v in r.items() if k not in ('kernel_rx','kernel_tx')})
"
