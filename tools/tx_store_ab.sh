# Tx field-store policy in the one-pass Tx (NETCSUM_TX_FIELD_STORE experiment builds build/txs1 =
# non-temporal, build/txs2 = system-scope write-through) against the in-tree library (one and two
# passes), 1 M x 1500-B IPv4/TCP, interleaved twice on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; T=${1:?tag}; O=gpurun_out; mkdir -p $O
export PS_NO_K2=1 PS_SPW=8 PS_NT=1 PS_D=4
for r in 1 2; do
  for v in default txs1 txs2; do
    lib=""; [ $v != default ] && lib=$R/uc-tcp-ip_amd/build/$v/libnetcsum_mi355x.so
    NETCSUM_LIB=$lib PS_PASSES=1,2 timeout -k 10 120 python tools/pkt_stream_probe.py > $O/${T}_${v}_$r.jsonl 2>> $O/${T}.err || { tail -5 $O/${T}.err; exit 1; }
  done
done
for f in $O/${T}_*.jsonl; do python -c "
import json
for l in open('$f'):
    d=json.loads(l); print('$f'.split('/')[-1], d['variant']['passes'], d['rx']['ms'], d['tx']['ms'], d['all_valid_after_tx'])"; done
