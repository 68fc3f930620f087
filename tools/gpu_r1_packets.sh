set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r1i_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r1i_gpu_tests.log; exit $rc
