set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out
for c in rx_s1500 rx_s1504; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    -d $O/r3h_${c}_im -o im --output-format csv -- python3 $R/tools/run_config.py $c 5 > $O/r3h_${c}_im.log 2>&1) || { tail -5 $O/r3h_${c}_im.log; exit 1; }
  grep "algo_bytes" $O/r3h_${c}_im.log
done
python3 tools/instmix_summary.py $O/r3h_rx_s1500_im $O/r3h_rx_s1504_im
