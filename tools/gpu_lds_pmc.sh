# One rocprofv3 --pmc pass of the SQ LDS / instruction counters over a BASELINE config
# (tools/run_config.py): LDS instructions, LDS-array cycles and bank-conflict cycles per launch,
# beside VALU instructions and busy cycles. usage (on the box): bash tools/gpu_lds_pmc.sh TAG CONFIG
set -o pipefail
T=${1:?tag}; C=${2:?config}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d $O/${T}_${C}_ldspmc -o lp --output-format csv -- python3 $R/tools/run_config.py $C 5 \
  > $O/${T}_${C}_ldspmc.log 2>&1 || { tail -5 $O/${T}_${C}_ldspmc.log; exit 1; }
tail -1 $O/${T}_${C}_ldspmc.log
