# rocprofv3 evidence for one BASELINE config (tools/run_config.py): --kernel-trace --stats, then
# SEPARATE --pmc passes for FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md §HBM: one TCC counter
# group per pass; FETCH_SIZE x2 for 16-B/lane streaming reads), summarised by tools/pmc_kernels.py.
# usage (on the box): [EXTRA_PMC="counters"] bash tools/gpu_pmc.sh TAG CONFIG [reps]
set -o pipefail
T=${1:?tag}; C=${2:?config}; N=${3:-30}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/${T}_${C}_trace -o trace --output-format csv \
  -- python3 $R/tools/run_config.py $C $N > $O/${T}_${C}_run.log 2>&1 || { tail -5 $O/${T}_${C}_run.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/${T}_${C}_fetch -o fetch --output-format csv \
  -- python3 $R/tools/run_config.py $C 5 > /dev/null 2> $O/${T}_${C}_fetch.err || { tail -5 $O/${T}_${C}_fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/${T}_${C}_write -o write --output-format csv \
  -- python3 $R/tools/run_config.py $C 5 > /dev/null 2> $O/${T}_${C}_write.err || { tail -5 $O/${T}_${C}_write.err; exit 1; }
if [ -n "$EXTRA_PMC" ]; then   # e.g. EXTRA_PMC="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum": one more pass
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $EXTRA_PMC -d $O/${T}_${C}_extra -o extra --output-format csv \
    -- python3 $R/tools/run_config.py $C 5 > /dev/null 2> $O/${T}_${C}_extra.err ) || { tail -5 $O/${T}_${C}_extra.err; exit 1; }
fi
cd $R && python3 tools/pmc_kernels.py $T $C $O > $O/${T}_${C}_pmc.json || exit 1
cat $O/${T}_${C}_run.log; cat $O/${T}_${C}_pmc.json
