# Round-1 measurement call: GPU tests, bench (default), smoke, secondary configs, rocprofv3 kernel
# trace + stats of bench.py, separate FETCH_SIZE / WRITE_SIZE PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r1h_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r1h_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r1h_bench.json 2> gpurun_out/r1h_bench.err || exit $?
cat gpurun_out/r1h_bench.json
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/r1h_configs.json 2> gpurun_out/r1h_configs.err || exit $?
cat gpurun_out/r1h_configs.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1h_trace -o trace --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/r1h_prof_bench.json 2> $R/gpurun_out/r1h_prof_trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_r1h_fetch -o fetch --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/r1h_pmc_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_r1h_write -o write --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/r1h_pmc_write.err || exit $?
echo done
