# Round-1 profiling call: geometry sweep, rocprofv3 kernel trace + stats of bench.py, and two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the same command (MI355X_MICROARCH.md §HBM).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python tools/sweep.py --c3 --c4 > gpurun_out/r1_sweep.jsonl 2> gpurun_out/r1_sweep.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1_trace -o trace --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/r1_prof_bench.json 2> $R/gpurun_out/r1_prof_trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_r1_fetch -o fetch --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/r1_pmc_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_r1_write -o write --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $R/gpurun_out/r1_pmc_write.err || exit $?
echo done
