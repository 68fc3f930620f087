set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python tools/sweep_align.py > gpurun_out/r1f_align.jsonl 2> gpurun_out/r1f_align.err || exit $?
echo done
