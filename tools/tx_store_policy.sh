# Tx finalize store cache-policy experiment: the default library and builds of netcsum_packets.hip
# with -DNETCSUM_TX_STORE_AUX=1/2/3/17 (sc0 / nt / sc0|nt / sc0|sc1) under uc-tcp-ip_amd/build/varN/
# (built on the CPU side beforehand). Each: oracle-sampled Tx, then timed (tools/tx_sweep.py).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
export TX_SWEEP_TILES=2 TX_SWEEP_NT=0,1 TX_SWEEP_GROUPS=0
timeout -k 10 120 python tools/tx_sweep.py > gpurun_out/r1sp_aux0.jsonl 2> gpurun_out/r1sp_aux0.err || exit $?
for A in 1 2 3 17; do
  NETCSUM_LIB=$R/uc-tcp-ip_amd/build/var$A/libnetcsum_mi355x.so timeout -k 10 120 python tools/tx_sweep.py > gpurun_out/r1sp_aux$A.jsonl 2> gpurun_out/r1sp_aux$A.err || exit $?
done
timeout -k 10 120 python tools/tx_sweep.py > gpurun_out/r1sp_aux0b.jsonl 2> gpurun_out/r1sp_aux0b.err || exit $?
head -50 gpurun_out/r1sp_aux*.jsonl
