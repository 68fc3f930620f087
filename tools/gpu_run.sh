# Parameterised GPU session (replaces round 1's one-off gpu_r1_*.sh scripts):
#   bash tools/gpu_run.sh TAG [tests|bench|prof|configs ...]   (default: tests bench prof)
# tests   full `-m gpu` suite                               -> gpurun_out/TAG_gpu_tests.log
# bench   driver-shaped bench (--gpus 1 --steps 20 --warmup 5) -> gpurun_out/TAG_bench.json
# prof    rocprofv3 --kernel-trace --stats of bench.py, then separate FETCH_SIZE / WRITE_SIZE PMC
#         passes (MI355X_MICROARCH.md §HBM), summarised   -> gpurun_out/TAG_pmc.json + TAG_trace/
# profc5  the same for the C5 shard (16 M segments)          -> gpurun_out/TAGc5_pmc.json
# configs tools/bench_configs.py (C1/C3/C4/packets/chains)  -> gpurun_out/TAG_configs.json
# Every GPU step has its own time limit; the first failure ends the session.
set -o pipefail
T=${1:?tag}; shift
STEPS=${*:-tests bench prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p $O
for s in $STEPS; do
  case $s in
  tests)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      > $O/${T}_gpu_tests.log 2>&1 || { tail -40 $O/${T}_gpu_tests.log; exit 1; }
    tail -2 $O/${T}_gpu_tests.log ;;
  bench)
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/${T}_bench.json 2> $O/${T}_bench.err \
      || { cat $O/${T}_bench.err; exit 1; }
    cat $O/${T}_bench.json ;;
  bench400)
    timeout -k 10 300 python bench.py > $O/${T}_bench400.json 2> $O/${T}_bench400.err || { cat $O/${T}_bench400.err; exit 1; }
    cat $O/${T}_bench400.json ;;
  c5)
    timeout -k 10 300 python bench.py --segments 16777216 --steps 50 --warmup 5 --no-cpu-baseline \
      > $O/${T}_c5_bench.json 2> $O/${T}_c5_bench.err || { cat $O/${T}_c5_bench.err; exit 1; }
    cat $O/${T}_c5_bench.json ;;
  prof)
    ( cd /tmp && export TMPDIR=/tmp &&
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}_trace -o trace --output-format csv \
        -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-c5-point --pmc off > $O/${T}_prof_bench.json 2> $O/${T}_prof_trace.err &&
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/${T}_fetch -o fetch --output-format csv \
        -- python3 $R/bench.py --steps 3 --warmup 1 --ramp-seconds 0 --no-cpu-baseline --no-c5-point --pmc off > /dev/null 2> $O/${T}_pmc_fetch.err &&
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/${T}_write -o write --output-format csv \
        -- python3 $R/bench.py --steps 3 --warmup 1 --ramp-seconds 0 --no-cpu-baseline --no-c5-point --pmc off > /dev/null 2> $O/${T}_pmc_write.err
    ) || { tail -20 $O/${T}_prof_trace.err $O/${T}_pmc_*.err; exit 1; }
    cat $O/${T}_prof_bench.json
    d() { dirname "$(find $O/${T}_$1 -name "$1_$2" -print -quit)"; }
    python tools/pmc_summary.py $T "$(d trace kernel_trace.csv)" "$(d fetch counter_collection.csv)" \
      "$(d write counter_collection.csv)" 1048576 $O/${T}_prof_bench.json $O > /dev/null || exit 1
    cp "$(d trace kernel_stats.csv)/trace_kernel_stats.csv" $O/${T}_rocprof_kernel_stats.csv
    python -c "import json;d=json.load(open('$O/${T}_pmc.json'));print({k:d.get(k) for k in ('dominant_kernel','rocprof_avg_us','traffic_over_algorithmic','kernel_src_sha')})" ;;
  profc5)   # the same evidence for the C5 shard (16 M segments per GPU): the summary bench.py --pmc file
            # uses for roofline.traffic at N > 1
    ( cd /tmp && export TMPDIR=/tmp && A="--segments 16777216 --no-cpu-baseline --pmc off" &&
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${T}c5_trace -o trace --output-format csv \
        -- python3 $R/bench.py --steps 30 --warmup 5 $A > $O/${T}c5_prof_bench.json 2> $O/${T}c5_prof_trace.err &&
      timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/${T}c5_fetch -o fetch --output-format csv \
        -- python3 $R/bench.py --steps 3 --warmup 1 --ramp-seconds 0 $A > /dev/null 2> $O/${T}c5_pmc_fetch.err &&
      timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/${T}c5_write -o write --output-format csv \
        -- python3 $R/bench.py --steps 3 --warmup 1 --ramp-seconds 0 $A > /dev/null 2> $O/${T}c5_pmc_write.err
    ) || { tail -20 $O/${T}c5_prof_trace.err $O/${T}c5_pmc_*.err; exit 1; }
    d() { dirname "$(find $O/${T}c5_$1 -name "$1_$2" -print -quit)"; }
    python tools/pmc_summary.py ${T}c5 "$(d trace kernel_trace.csv)" "$(d fetch counter_collection.csv)" \
      "$(d write counter_collection.csv)" 16777216 $O/${T}c5_prof_bench.json $O > /dev/null || exit 1
    cp "$(d trace kernel_stats.csv)/trace_kernel_stats.csv" $O/${T}c5_rocprof_kernel_stats.csv
    python -c "import json;d=json.load(open('$O/${T}c5_pmc.json'));print({k:d.get(k) for k in ('dominant_kernel','rocprof_avg_us','traffic_over_algorithmic','kernel_src_sha')})" ;;
  configs)
    timeout -k 10 400 python tools/bench_configs.py > $O/${T}_configs.json 2> $O/${T}_configs.err || { tail -20 $O/${T}_configs.err; exit 1; }
    cat $O/${T}_configs.json ;;
  smoke)
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
  *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session $T done"
