# tools/c2_probe.py under experiment builds of the library (uc-tcp-ip_amd/build/<name>, made with
# make OUT=build/<name> LIB=build/<name>/libnetcsum_mi355x.so EXTRA=-D...): VARIANTS names them,
# "default" is the in-tree library. Usage on the box: VARIANTS="default st1" bash tools/c2_variants.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; T=${1:-r2cv}
for v in ${VARIANTS:-default}; do
  lib=""; [ $v != default ] && lib=$R/uc-tcp-ip_amd/build/$v/libnetcsum_mi355x.so
  echo "== $v"
  NETCSUM_LIB=$lib timeout -k 10 200 python tools/c2_probe.py > gpurun_out/${T}_$v.jsonl 2> gpurun_out/${T}_$v.err || { tail -3 gpurun_out/${T}_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/${T}_$v.jsonl'):
    d=json.loads(l); print(d['variant'], d['ms_med'], d['GBps_med'])"
done
