timeout -k 10 300 python -u -m pytest tests/test_gpu_pktstream.py tests/test_gpu_packets.py tests/test_gpu_hdr_waits.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r2ps_tests.log 2>&1; rc=$?; tail -25 gpurun_out/r2ps_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/pkt_stream_probe.py > gpurun_out/r2ps_probe.jsonl 2> gpurun_out/r2ps_probe.err || { tail -3 gpurun_out/r2ps_probe.err; exit 1; }
cat gpurun_out/r2ps_probe.jsonl
timeout -k 10 300 python tools/c3_sweep.py > gpurun_out/r2ps_c3_sweep.jsonl 2> gpurun_out/r2ps_c3_sweep.err || { tail -3 gpurun_out/r2ps_c3_sweep.err; exit 1; }
cat gpurun_out/r2ps_c3_sweep.jsonl
bash tools/gpu_pmc.sh r2ps c3 && bash tools/gpu_pmc.sh r2ps tx && bash tools/gpu_pmc.sh r2ps tx2
