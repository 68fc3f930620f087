#!/bin/bash
# Round-4: is the 2-KiB-slot ring's 1.11 x read traffic the L2 line size or the non-temporal load
# policy? FETCH_SIZE (and L2->HBM read requests by size) of Rx with the default nt stream loads and
# with plain loads (NETCSUM_TUNE_NT_LOADS 0), 2-KiB slots and the mixed ring.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for c in rx_nb2k rx_nb2k.nt0 rx_ring.nt0; do
  EXTRA_PMC="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_128B_sum" bash tools/gpu_pmc.sh r4t $c > /dev/null || exit 1
done
python3 - <<'PY'
import json
for c in ("rx_nb2k", "rx_nb2k.nt0", "rx_ring.nt0"):
    d = json.load(open(f"gpurun_out/r4t_{c}_pmc.json"))
    for k, v in d["kernels"].items():
        if "pkt_stream_kernel" in k:
            print(c, k[60:110], v["avg_us"], v["traffic_over_algorithmic"], {x: v.get(x) for x in v if x.startswith("TCC")})
PY
