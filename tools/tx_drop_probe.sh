# Tx finalize: is the cost the memory-side effect of the field writes? Compare the default library
# with a build whose field stores are all out of range (-DNETCSUM_TX_DROP_STORES: identical
# instructions, the hardware drops every store): timing (tx_sweep) + PMC passes (wave lifetime, L2
# fabric requests). Build uc-tcp-ip_amd/build/vardrop on the CPU side first.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
D=$R/uc-tcp-ip_amd/build/vardrop/libnetcsum_mi355x.so
export TX_SWEEP_TILES=2 TX_SWEEP_NT=0 TX_SWEEP_GROUPS=0
timeout -k 10 120 python tools/tx_sweep.py > gpurun_out/r1dp_default.jsonl 2> gpurun_out/r1dp_default.err || exit $?
NETCSUM_LIB=$D timeout -k 10 120 python tools/tx_sweep.py > gpurun_out/r1dp_drop.jsonl 2> gpurun_out/r1dp_drop.err || exit $?
cat gpurun_out/r1dp_default.jsonl gpurun_out/r1dp_drop.jsonl
cd /tmp && export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
B="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
i=0
for cfg in "default rx" "default tx" "drop tx"; do
  set -- $cfg
  lib=""; [ "$1" = drop ] && lib=$D
  for S in "$A" "$B"; do
    i=$((i+1))
    NETCSUM_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $S -d $R/gpurun_out/pmc_r1dp_${1}_${2}_$i -o pmc --output-format csv -- python3 $R/tools/run_pkt_variant.py $2 30 > $R/gpurun_out/pmc_r1dp_${1}_${2}_$i.log 2>&1 || exit $?
  done
done
echo done
