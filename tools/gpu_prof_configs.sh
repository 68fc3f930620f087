# rocprofv3 kernel trace + stats of tools/bench_configs.py (secondary configs: C3, C4, Rx, Tx, chains,
# host path, drop-in): per-kernel durations backing DESIGN.md §9's table.
set -o pipefail
T=${1:-r1cfg}
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T:-r1cfg} -o cfg --output-format csv -- python3 $R/tools/bench_configs.py > $R/gpurun_out/${T:-r1cfg}_configs.json 2> $R/gpurun_out/${T:-r1cfg}.err || exit $?
echo done
