# Header-kernel bring-up: its parity tests first (stop on failure), then the C3 sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "small_aligned" > gpurun_out/r1h_hdr_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r1h_hdr_tests.log; [ $rc -eq 0 ] || exit $rc
SWEEP_C3=1 SWEEP_C3_SPEC=${SPEC:-2,3:1:1,2,4} timeout -k 10 400 python -u tools/sweep_stream.py 3 > gpurun_out/r1h_c3_sweep.jsonl 2> gpurun_out/r1h_c3_sweep.err || exit $?
cat gpurun_out/r1h_c3_sweep.jsonl
