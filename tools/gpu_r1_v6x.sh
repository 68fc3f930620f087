# IPv6 extreme-size packet tests only.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_packets_v6.py tests/test_gpu_packets.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r1v4x_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r1v4x_gpu_tests.log; exit $rc
