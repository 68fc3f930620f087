set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1tx2p -o tr --output-format csv -- python3 $R/tools/run_pkt_variant.py tx 300 wb=3 nt=1 tile=2 > $R/gpurun_out/r1tx2p_prof.log 2>&1 || exit $?
echo done
