# Per-call drop-in path (completion-word polling): the GPU parity suite (most of it goes through the
# drop-in functions), then the config bench (C1_dropin_call_us).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r1c1_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r1c1_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_configs.py > gpurun_out/r1c1_configs.json 2> gpurun_out/r1c1_configs.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/r1c1_configs.json'));print(d['C1_dropin_call_us'])"
