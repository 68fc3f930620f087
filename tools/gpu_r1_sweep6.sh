set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r1g_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r1g_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/sweep.py --c3 --c4 > gpurun_out/r1g_sweep.jsonl 2> gpurun_out/r1g_sweep.err || exit $?
echo sweep-done
