# Round-1 measurement call: GPU tests, smoke, bench (default), secondary configs, rocprofv3 kernel
# trace + stats of bench.py, separate FETCH_SIZE / WRITE_SIZE PMC passes. Usage: bash ... <tag>
set -o pipefail
T=${1:-r1s}
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/${T}_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
cat gpurun_out/${T}_bench.json
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/${T}_configs.json 2> gpurun_out/${T}_configs.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_trace -o trace --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/${T}_prof_bench.json 2> $R/gpurun_out/${T}_prof_trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_${T}_fetch -o fetch --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/${T}_pmc_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_${T}_write -o write --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/${T}_pmc_write.err || exit $?
echo done
