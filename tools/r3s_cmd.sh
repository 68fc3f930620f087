# Round-3 session-2 GPU call: the restored tree's suite / smoke / bench / profile, then two probes
# (Tx write-back forms, fragment buffer pitch). usage (on the box): bash tools/r3s_cmd.sh TAG [steps]
set -o pipefail
T=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p $O
STEPS=${*:-base wb pitch}
for s in $STEPS; do
  case $s in
  base)
    bash tools/gpu_run.sh $T tests smoke bench prof || exit 1 ;;
  wb)
    timeout -k 10 180 tools/build/tx_wb_probe 1500 > $O/${T}_tx_wb_probe.jsonl 2>&1 || { tail -5 $O/${T}_tx_wb_probe.jsonl; exit 1; }
    timeout -k 10 180 tools/build/tx_wb_probe 1520 >> $O/${T}_tx_wb_probe.jsonl 2>&1 || { tail -5 $O/${T}_tx_wb_probe.jsonl; exit 1; }
    cat $O/${T}_tx_wb_probe.jsonl ;;
  wb1500)
    timeout -k 10 180 tools/build/tx_wb_probe 1500 > $O/${T}_tx_wb_probe.jsonl 2>&1 || { tail -5 $O/${T}_tx_wb_probe.jsonl; exit 1; }
    cat $O/${T}_tx_wb_probe.jsonl ;;
  c3ceil)
    timeout -k 10 180 python -u tools/c3_ceiling_probe.py > $O/${T}_c3_ceiling.jsonl 2>&1 || { tail -5 $O/${T}_c3_ceiling.jsonl; exit 1; }
    cat $O/${T}_c3_ceiling.jsonl ;;
  pkttests)
    timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      tests/test_gpu_pktstream.py tests/test_gpu_packets.py tests/test_gpu_offload.py tests/test_gpu_host.py -m gpu \
      > $O/${T}_pkt_tests.log 2>&1 || { tail -30 $O/${T}_pkt_tests.log; exit 1; }
    tail -2 $O/${T}_pkt_tests.log ;;
  txsec)
    timeout -k 10 400 python -u tools/tx_sector_probe.py > $O/${T}_tx_sector_probe.jsonl 2>&1 || { tail -5 $O/${T}_tx_sector_probe.jsonl; exit 1; }
    python3 -c "
import json
for l in open('$O/${T}_tx_sector_probe.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print({k:v for k,v in r.items() if k!='kernel'})
" ;;
  frag)
    timeout -k 10 300 python -u tools/frag_stream_probe.py > $O/${T}_frag_stream_probe.jsonl 2>&1 || { tail -5 $O/${T}_frag_stream_probe.jsonl; exit 1; }
    python3 -c "
import json
for l in open('$O/${T}_frag_stream_probe.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print({k:v for k,v in r.items() if not k.startswith('kernel')})
" ;;
  pitch)
    timeout -k 10 300 python -u tools/pitch_probe.py > $O/${T}_pitch_probe.jsonl 2>&1 || { tail -5 $O/${T}_pitch_probe.jsonl; exit 1; }
    python3 -c "
import json
for l in open('$O/${T}_pitch_probe.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print({k:v for k,v in r.items() if not k.startswith('kernel')})
" ;;
  *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "r3s session $T done"
