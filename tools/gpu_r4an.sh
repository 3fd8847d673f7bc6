# float64 grid rule (largest grid under the cap instead of halving): f64 tests and C5 / C3 timing
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4an; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_blobs.py::test_float64_input_identical_to_reference "tests/test_gpu_api.py::test_corr_csv_configs" tests/test_gpu_api.py::test_auto_precision_float64_input_is_f64 "tests/test_gpu_kmeans.py::test_f64_labels_match_sklearn_float64" "tests/test_gpu_kmeans.py::test_f64_relocation_with_ties_is_pinned" tests/test_gpu_fit.py -q --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
for c in "c5 64" "c3 128" "c2 500"; do
  set -- $c
  timeout -k 10 400 python -u tools/f64_time.py $1 $2 2>&1 | grep -v amdgpu | tee -a $O/f64_vs_fast.txt || exit 1
done
