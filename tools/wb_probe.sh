# Tx write-cost probe (DESIGN §9 Tx row): the C2 stream kernel alone vs builds that add in-place
# field writes at +10/+36 of every segment (NETCSUM_STREAM_WB_PROBE 1: 2-byte writes as one burst
# per wave after its run; 2: as soon as each segment's last byte is read; 3: whole aligned 64-B
# lines, burst). Build the variants first (uc-tcp-ip_amd/build/wbN, make EXTRA=-DNETCSUM_STREAM_WB_PROBE=N).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; T=${1:-r2wb}
for v in ${VARIANTS:-default wb1 wb2 wb3 default}; do
  lib=""; [ $v != default ] && lib=$R/uc-tcp-ip_amd/build/$v/libnetcsum_mi355x.so
  NETCSUM_LIB=$lib timeout -k 10 120 python bench.py $BENCH_ARGS --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${T}_$v.json'));r=d['roofline'];print('$v', r['kernel_ms'], r['kernel_ms_median'], d['ms_per_step'], d['parity_sample_ok'])"
done
if [ -z "$NO_TX" ]; then
  timeout -k 10 120 python tools/tx_sweep.py > gpurun_out/${T}_tx_sweep.jsonl 2> gpurun_out/${T}_tx_sweep.err || exit 1
  cat gpurun_out/${T}_tx_sweep.jsonl
fi
