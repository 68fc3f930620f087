export PS_SPW=8,16 PS_NT=1 PS_D=4,8 PS_PASSES=1,2
timeout -k 10 300 python tools/pkt_stream_probe.py > gpurun_out/r2tx_probe.jsonl 2> gpurun_out/r2tx_probe.err || { tail -3 gpurun_out/r2tx_probe.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r2tx_probe.jsonl'):
    d=json.loads(l); print(d['variant'], d['rx']['ms'], d['tx']['ms'], d['all_valid_after_tx'])"
timeout -k 10 200 python -u -m pytest tests/test_gpu_pktstream.py tests/test_gpu_hdrstream.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2tx_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r2tx_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/c3_sweep.py > gpurun_out/r2tx_c3_sweep.jsonl 2> gpurun_out/r2tx_c3_sweep.err || { tail -3 gpurun_out/r2tx_c3_sweep.err; exit 1; }
cat gpurun_out/r2tx_c3_sweep.jsonl
