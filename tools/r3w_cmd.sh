# Round-3 A/B sessions: the product library (A) against experiment / previous builds in
# uc-tcp-ip_amd/build/var*/ (NETCSUM_LIB), same box, interleaved. Env: VARS (default "B C"),
# CFG (tools/run_config.py config, default chains), TESTS (pytest files run against each variant
# first, default tests/test_gpu_chains.py), O (output dir, default gpurun_out/r3w).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=${O:-$R/gpurun_out/r3w}; mkdir -p $O; cd $R
P=$R/uc-tcp-ip_amd/libnetcsum_mi355x.so
for v in ${VARS:-B C}; do
  NETCSUM_LIB=$R/uc-tcp-ip_amd/build/var$v/libnetcsum_mi355x.so timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_chains.py} -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; exit 1; }
done
for rep in 1 2 3; do
  for v in A ${VARS:-B C}; do
    L=$P; [ $v = A ] || L=$R/uc-tcp-ip_amd/build/var$v/libnetcsum_mi355x.so
    echo "== rep $rep var $v" >> $O/ab.log
    NETCSUM_LIB=$L timeout -k 10 120 python3 tools/run_config.py ${CFG:-chains} 300 >> $O/ab.log 2>&1 || { echo "run $v failed"; exit 1; }
  done
done
echo done
