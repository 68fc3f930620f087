set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python -m pytest tests/test_gpu_packets.py tests/test_gpu_chains.py -x -q -p no:cacheprovider > gpurun_out/r1l_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r1l_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/r1l_configs.json 2> gpurun_out/r1l_configs.err || exit $?
cat gpurun_out/r1l_configs.json
