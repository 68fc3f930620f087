# Run one measurement tool under experiment builds of the library (uc-tcp-ip_amd/build/<name>, made
# with make OUT=build/<name> LIB=build/<name>/libnetcsum_mi355x.so EXTRA=-D...); "default" is the
# in-tree library. The tool's own env knobs pass through.
# Usage on the box: VARIANTS="default hsp" bash tools/lib_variants.sh TAG tools/c3_sweep.py
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; T=${1:?tag}; TOOL=${2:?tool}
for v in ${VARIANTS:-default}; do
  lib=""; [ $v != default ] && lib=$R/uc-tcp-ip_amd/build/$v/libnetcsum_mi355x.so
  echo "== $v"
  NETCSUM_LIB=$lib timeout -k 10 200 python $TOOL > gpurun_out/${T}_$v.jsonl 2> gpurun_out/${T}_$v.err || { tail -3 gpurun_out/${T}_$v.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/${T}_$v.jsonl'):
    d=json.loads(l); print(d['variant'], d.get('ms_med', d.get('ms')), d.get('GBps_med', d.get('GBps_algo', d.get('GBps'))))"
done
