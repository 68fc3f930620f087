# PMC comparison of fused Rx vs Tx finalize: one rocprofv3 --pmc pass per (variant, counter set).
# Usage: bash tools/gpu_pmc_pkt.sh <tag>
set -o pipefail
T=$1
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY"
S2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
for v in "rx" "tx" "tx wb=1" "tx nt=0 tile=2"; do
  tag=$(echo "$v" | tr ' =' '__')
  i=0
  for S in "$S1" "$S2" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $S -d $R/gpurun_out/pmc_${T}_${tag}_$i -o pmc --output-format csv -- python3 $R/tools/run_pkt_variant.py $v 30 > $R/gpurun_out/pmc_${T}_${tag}_$i.log 2>&1 || exit $?
  done
done
echo done
