# C3: seg_hdr_kernel with its 33.5 MB of result stores dropped (same instructions, offsets out of
# range) vs the default build, plus the FETCH/WRITE PMC of the default C3 launch.
for v in default hd; do
  lib=""; [ $v != default ] && lib=$GRAFT_REPO_ROOT/uc-tcp-ip_amd/build/$v/libnetcsum_mi355x.so
  NETCSUM_LIB=$lib timeout -k 10 120 python tools/run_config.py c3 200 || exit 1
done
NETCSUM_LIB=$GRAFT_REPO_ROOT/uc-tcp-ip_amd/build/hd/libnetcsum_mi355x.so timeout -k 10 120 python tools/run_config.py c3 200 || exit 1
timeout -k 10 120 python tools/run_config.py c3 200 || exit 1
bash tools/gpu_pmc.sh r2hd c3 > /dev/null && python -c "
import json;d=json.load(open('gpurun_out/r2hd_c3_pmc.json'))
for k,v in d['kernels'].items():
    if 'hdr' in k: print(k[:70], v)"
