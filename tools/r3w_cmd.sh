# Round-3 chain-pass-1 A/B session: the product library (A) against experiment builds of
# netcsum_chains.hip in uc-tcp-ip_amd/build/var*/ (NETCSUM_LIB), same box, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3w; mkdir -p $O; cd $R
P=$R/uc-tcp-ip_amd/libnetcsum_mi355x.so
for v in ${VARS:-B C}; do
  NETCSUM_LIB=$R/uc-tcp-ip_amd/build/var$v/libnetcsum_mi355x.so timeout -k 10 300 python -u -m pytest tests/test_gpu_chains.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; exit 1; }
done
for rep in 1 2 3; do
  for v in A ${VARS:-B C}; do
    L=$P; [ $v = A ] || L=$R/uc-tcp-ip_amd/build/var$v/libnetcsum_mi355x.so
    echo "== rep $rep var $v" >> $O/ab.log
    NETCSUM_LIB=$L timeout -k 10 120 python3 tools/run_config.py chains 300 >> $O/ab.log 2>&1 || { echo "run $v failed"; exit 1; }
  done
done
echo done
