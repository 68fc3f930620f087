set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r1p_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r1p_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/sweep.py --c3 --c4 > gpurun_out/r1p_sweep.jsonl 2> gpurun_out/r1p_sweep.err || exit $?
timeout -k 10 300 python tools/rx_sweep.py > gpurun_out/r1p_rx_sweep.jsonl 2> gpurun_out/r1p_rx_sweep.err || exit $?
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/r1p_configs.json 2> gpurun_out/r1p_configs.err || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r1p_bench.json 2> gpurun_out/r1p_bench.err || exit $?
cat gpurun_out/r1p_configs.json gpurun_out/r1p_bench.json
