set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r1v_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r1v_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sweep.py --no-c2 --c3 > gpurun_out/r1v_sweep.jsonl 2> gpurun_out/r1v_sweep.err || exit $?
cat gpurun_out/r1v_sweep.jsonl
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/r1v_configs.json 2> gpurun_out/r1v_configs.err || exit $?
cat gpurun_out/r1v_configs.json
