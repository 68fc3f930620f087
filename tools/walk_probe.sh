# Walk pass (pkt_v6_walk_kernel) cost: IPv6 / mixed / IPv4 probes (no chain to walk), then the worst
# case (every IPv6 datagram behind a 200-B Destination Options header), with a rocprof kernel trace.
set -o pipefail
O=gpurun_out; mkdir -p $O; T=${1:-r2zs}
export PS_NO_K2=1 PS_NT=1 PS_D=4 PS_PASSES=2
PS_VER=6 PS_SPW=8 timeout -k 10 120 python tools/pkt_stream_probe.py > $O/${T}_walk_v6.jsonl 2>$O/${T}_walk.err &&
PS_VER=mix PS_SPW=16 timeout -k 10 120 python tools/pkt_stream_probe.py > $O/${T}_walk_mix.jsonl 2>>$O/${T}_walk.err &&
PS_VER=4 PS_SPW=8 timeout -k 10 120 python tools/pkt_stream_probe.py > $O/${T}_walk_v4.jsonl 2>>$O/${T}_walk.err &&
PS_CHAIN=1 PS_VER=6 PS_SPW=8 timeout -k 10 120 python tools/pkt_stream_probe.py > $O/${T}_walk_v6chain.jsonl 2>>$O/${T}_walk.err &&
( cd /tmp && export TMPDIR=/tmp && PS_CHAIN=1 PS_VER=6 PS_SPW=8 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/$O/${T}_walk_trace -o t --output-format csv -- python3 $R/tools/pkt_stream_probe.py > /dev/null 2>>$R/$O/${T}_walk.err ) &&
cat $O/${T}_walk_*.jsonl && cat $(find $O/${T}_walk_trace -name 't_kernel_stats.csv') | cut -c1-200
