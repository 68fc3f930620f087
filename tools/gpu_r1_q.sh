set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python bench.py > gpurun_out/r1q_bench.json 2> gpurun_out/r1q_bench.err || exit $?
timeout -k 10 300 python bench.py --tune group=32 > gpurun_out/r1q_bench_g32.json 2> gpurun_out/r1q_bench_g32.err || exit $?
cat gpurun_out/r1q_bench.json gpurun_out/r1q_bench_g32.json
