set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1tx3 -o tr --output-format csv -- python3 $R/tools/run_pkt_variant.py tx 30 wb=3 nt=1 tile=2 > $R/gpurun_out/r1tx3_prof.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1tx0 -o tr --output-format csv -- python3 $R/tools/run_pkt_variant.py tx 30 wb=0 nt=0 tile=2 > $R/gpurun_out/r1tx0_prof.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1rx -o tr --output-format csv -- python3 $R/tools/run_pkt_variant.py rx 30 > $R/gpurun_out/r1rx_prof.log 2>&1 || exit $?
echo done
