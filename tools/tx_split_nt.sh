# Tx finalize: header slot plain + remaining chunks non-temporal (-DNETCSUM_TX_SPLIT_NT=1 build under
# uc-tcp-ip_amd/build/varsplit) vs the default (all plain), both timed by tools/tx_sweep.py (nt=0).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
export TX_SWEEP_TILES=2,4 TX_SWEEP_NT=0 TX_SWEEP_GROUPS=0
timeout -k 10 120 python tools/tx_sweep.py > gpurun_out/r1sn_default.jsonl 2> gpurun_out/r1sn_default.err || exit $?
NETCSUM_LIB=$R/uc-tcp-ip_amd/build/varsplit/libnetcsum_mi355x.so timeout -k 10 120 python tools/tx_sweep.py > gpurun_out/r1sn_split.jsonl 2> gpurun_out/r1sn_split.err || exit $?
timeout -k 10 120 python tools/tx_sweep.py > gpurun_out/r1sn_default2.jsonl 2> gpurun_out/r1sn_default2.err || exit $?
cat gpurun_out/r1sn_default.jsonl gpurun_out/r1sn_split.jsonl gpurun_out/r1sn_default2.jsonl
