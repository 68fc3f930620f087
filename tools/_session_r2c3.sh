timeout -k 10 300 python tools/c3_sweep.py > gpurun_out/r2c3b_sweep.jsonl 2> gpurun_out/r2c3b_sweep.err || { tail -3 gpurun_out/r2c3b_sweep.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r2c3b_sweep.jsonl'):
    d=json.loads(l); print(d.get('variant'), d.get('ms'), d.get('GBps_algo', d.get('GBps')), d.get('same'))"
timeout -k 10 300 python -u -m pytest tests/test_gpu_hdrstream.py tests/test_gpu_hdr_waits.py tests/test_gpu_configs_full.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2c3b_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r2c3b_tests.log; exit $rc
