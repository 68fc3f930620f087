set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 500 python tools/sweep.py --c3 --c4 > gpurun_out/r1o_sweep.jsonl 2> gpurun_out/r1o_sweep.err || exit $?
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/r1o_configs.json 2> gpurun_out/r1o_configs.err || exit $?
cat gpurun_out/r1o_configs.json
