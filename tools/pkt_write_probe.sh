# Where does the Tx record pass lose time against Rx? (DESIGN §9 Tx row) The same 1 M x 1500-B batch
# timed with experiment builds of the run-stream packet kernel (NETCSUM_PKTSTREAM_PROBE: 1 Rx stores
# nothing, 2 Rx stores 8 B per packet, 4 Tx record pass stores nothing, 5 Tx records into the probe's
# torch buffer, 6 Tx 4-B records) next to the default build (PW_VARIANTS picks the builds).
# Build first: make -C uc-tcp-ip_amd OUT=build/psN LIB=build/psN/libnetcsum_mi355x.so EXTRA=-DNETCSUM_PKTSTREAM_PROBE=N
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; T=${1:-r2pw}
export PS_SPW=8,16 PS_NT=1 PS_D=4 PS_PASSES=1,2 PS_TX_FLAGS=1
for v in ${PW_VARIANTS:-default ps1 ps2 ps4}; do
  lib=""; [ $v != default ] && lib=$R/uc-tcp-ip_amd/build/$v/libnetcsum_mi355x.so
  echo "== $v"
  NETCSUM_LIB=$lib timeout -k 10 200 python tools/pkt_stream_probe.py > gpurun_out/${T}_$v.jsonl 2> gpurun_out/${T}_$v.err || { tail -3 gpurun_out/${T}_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/${T}_$v.jsonl'):
    d=json.loads(l); print(d['variant'], d['rx']['ms'], d['tx']['ms'])"
done
