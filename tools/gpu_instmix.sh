# One rocprofv3 --pmc pass of SQ instruction / cycle counters over a BASELINE config
# (tools/run_config.py): dynamic VALU / SALU / VMEM instructions and wave cycles per launch.
# usage (on the box): bash tools/gpu_instmix.sh TAG CONFIG   -> gpurun_out/TAG_CONFIG_instmix/
set -o pipefail
T=${1:?tag}; C=${2:?config}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d $O/${T}_${C}_instmix -o im --output-format csv -- python3 $R/tools/run_config.py $C 5 \
  > $O/${T}_${C}_instmix.log 2>&1 || { tail -5 $O/${T}_${C}_instmix.log; exit 1; }
tail -1 $O/${T}_${C}_instmix.log
