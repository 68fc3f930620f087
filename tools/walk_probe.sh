set -o pipefail
O=gpurun_out; mkdir -p $O
export PS_NO_K2=1 PS_NT=1 PS_D=4 PS_PASSES=2
PS_VER=6 PS_SPW=8 timeout -k 10 120 python tools/pkt_stream_probe.py > $O/r2zs_walk_v6.jsonl 2>$O/r2zs_walk.err &&
PS_VER=mix PS_SPW=16 timeout -k 10 120 python tools/pkt_stream_probe.py > $O/r2zs_walk_mix.jsonl 2>>$O/r2zs_walk.err &&
PS_VER=4 PS_SPW=8 timeout -k 10 120 python tools/pkt_stream_probe.py > $O/r2zs_walk_v4.jsonl 2>>$O/r2zs_walk.err &&
( cd /tmp && export TMPDIR=/tmp && PS_VER=6 PS_SPW=8 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/$O/r2zs_walk_trace -o t --output-format csv -- python3 $R/tools/pkt_stream_probe.py > /dev/null 2>>$R/$O/r2zs_walk.err ) &&
cat $O/r2zs_walk_*.jsonl && cat $(find $O/r2zs_walk_trace -name 't_kernel_stats.csv') | cut -c1-200
