# CRC-32 11-bit-table lookups split between LDS and the vector-memory path (NETCSUM_CRC_L1_SPLIT
# experiment builds build/l1s1, build/l1s2) against the in-tree library, one box, crc_probe on
# 1500 / 9000 / 300-B frames and the varlen batch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; T=${1:?tag}; O=gpurun_out; mkdir -p $O
for v in default l1s1 l1s2; do
  lib=""; [ $v != default ] && lib=$R/uc-tcp-ip_amd/build/$v/libnetcsum_mi355x.so
  NETCSUM_LIB=$lib timeout -k 10 240 python tools/crc_probe.py 2 1500,9000,300 > $O/${T}_$v.jsonl 2> $O/${T}_$v.err || { tail -5 $O/${T}_$v.err; exit 1; }
done
