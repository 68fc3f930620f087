# Roofline evidence for every DESIGN.md §9 row (tools/gpu_pmc.sh per config: kernel trace +
# FETCH_SIZE / WRITE_SIZE passes; the Tx rows also the L2 write-request counters), then the
# configs record (tools/bench_configs.py). usage (on the box): bash tools/gpu_pmc_all.sh TAG [configs...]
set -o pipefail
T=${1:?tag}; shift
CONFIGS=${*:-c3 c4 pool1520 pool1520mix pool2k pool2kmix chains rx rx6 rxmix rxb txb tx tx_nb rx_nb tx_nb2k rx_nb2k rx_nb2kv tx_nb2kv rx_ring tx_ring rx_ringv tx_ringv}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
for c in $CONFIGS; do
  case $c in
    tx|tx_nb|tx_nb2k|txb|tx_ring|tx_ringv|tx_nb2kv) X="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" ;;
    *) X="" ;;
  esac
  EXTRA_PMC="$X" bash tools/gpu_pmc.sh $T $c > gpurun_out/${T}_${c}_session.log 2>&1 || { tail -20 gpurun_out/${T}_${c}_session.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${T}_${c}_pmc.json'));print('$c', {k:(v.get('avg_us'),v.get('traffic_over_algorithmic')) for k,v in d['kernels'].items()})"
done
