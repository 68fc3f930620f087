set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 200 python tools/launch_probe.py > gpurun_out/r1r_launch.json 2> gpurun_out/r1r_launch.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r1r_bench_a.json 2> gpurun_out/r1r_bench_a.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/r1r_bench_b.json 2> gpurun_out/r1r_bench_b.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --tune group=32 > gpurun_out/r1r_bench_c.json 2> gpurun_out/r1r_bench_c.err || exit $?
cat gpurun_out/r1r_launch.json gpurun_out/r1r_bench_a.json gpurun_out/r1r_bench_b.json gpurun_out/r1r_bench_c.json
