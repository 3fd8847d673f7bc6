# manhattan variant (float64 staged in LDS) against the current kernel: exactness test, then
# timings at n = 20 000 (digest of a row sample must agree).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4w; mkdir -p $O
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/consensus_clustering_amd
CCMI_LIB=$L/libccmi_pr_f64lds.so timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py::test_manhattan_kernel_matches_scipy -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/test.log 2>&1
rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || exit $rc
for lib in pr_base pr_f64lds pr_base pr_f64lds; do
  CCMI_LIB=$L/libccmi_$lib.so timeout -k 10 200 python -u tools/manhattan_time.py 20000 2 2>&1 | grep -v amdgpu | tee -a $O/ab.txt || exit 1
done
