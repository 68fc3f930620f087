# A/B of the C5 shard (16 M x 1500 B) between the in-tree library and an experiment build on ONE box:
#   bash tools/c5_ab.sh TAG LIB   (interleaved: A B A B)
set -o pipefail
T=${1:?tag}; L=${2:?lib}; O=gpurun_out; mkdir -p $O
A="--segments 16777216 --steps 30 --warmup 5 --no-cpu-baseline --pmc off"
for r in 1 2; do
  timeout -k 10 200 python bench.py $A > $O/${T}_cur_$r.json 2>>$O/${T}.err || exit 1
  NETCSUM_LIB=$L timeout -k 10 200 python bench.py $A > $O/${T}_alt_$r.json 2>>$O/${T}.err || exit 1
done
for f in $O/${T}_*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f',d['ms_per_step'],d['roofline']['kernel_ms'])"; done
