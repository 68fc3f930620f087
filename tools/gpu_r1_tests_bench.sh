set -o pipefail
cd $GRAFT_REPO_ROOT
echo "host: $(hostname) cpus=$(nproc)"; rocm-smi --showproductname 2>/dev/null | head -8
timeout -k 10 800 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r1_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r1_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r1_bench.json 2> gpurun_out/r1_bench.err
rc=$?; cat gpurun_out/r1_bench.json; tail -3 gpurun_out/r1_bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()"
