# Varlen stream kernel: parity tests (stop on failure), then the C4 sweep (packed and NIC-ring layouts).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "varlen or small_aligned or stream" > gpurun_out/r1z_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r1z_tests.log; [ $rc -eq 0 ] || exit $rc
SWEEP_C4=1 SWEEP_C4_SPEC="4:16,32" timeout -k 10 400 python -u tools/sweep_stream.py 3 > gpurun_out/r1z_c4_sweep.jsonl 2> gpurun_out/r1z_c4_sweep.err || exit $?
SWEEP_C4=1 SWEEP_C4_RING=1 SWEEP_C4_SPEC="4:8,16" timeout -k 10 400 python -u tools/sweep_stream.py 3 > gpurun_out/r1z_c4ring_sweep.jsonl 2> gpurun_out/r1z_c4ring_sweep.err || exit $?
cat gpurun_out/r1z_c4_sweep.jsonl gpurun_out/r1z_c4ring_sweep.jsonl
