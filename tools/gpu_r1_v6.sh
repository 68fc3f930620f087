# IPv6 packet batches: GPU parity (v6 and the unchanged v4 packet tests), then the config bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_packets_v6.py tests/test_gpu_packets.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r1v6d_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r1v6d_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/r1v6d_configs.json 2> gpurun_out/r1v6d_configs.err || exit $?
cat gpurun_out/r1v6d_configs.json
