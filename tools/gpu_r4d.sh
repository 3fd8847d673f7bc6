# Staged co-sampling counts in the co-association epilogue: correctness (co-association tests,
# the full-size tile checks, the f64 relocation test) and per-K timings against the previous
# library (libccmi_co_base.so) at C5, C2 and C3.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4d; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_coassoc.py tests/test_gpu_scale.py::test_c5_full_size tests/test_gpu_scale.py::test_c2_full_size_with_matrices "tests/test_gpu_kmeans.py::test_f64_relocation_with_ties_is_pinned" tests/test_gpu_api.py tests/test_gpu_dist.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|f64 relocation" $O/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
for c in c5 c2 c3; do
  timeout -k 10 200 python -u tools/co_only.py $c > $O/co_$c.txt 2>&1 || exit $?
  CCMI_LIB=consensus_clustering_amd/libccmi_co_base.so timeout -k 10 200 python -u tools/co_only.py $c > $O/co_${c}_base.txt 2>&1 || exit $?
  echo "== $c staged"; grep -v amdgpu.ids $O/co_$c.txt | tail -2
  echo "== $c base"; grep -v amdgpu.ids $O/co_${c}_base.txt | tail -2
done
