# float64 k-means with the fragment row image: throughput at C3 / C5 under 40 and 96 GB budgets
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4ak; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/f64_budget.py c3 128 40 96 20 2>&1 | grep -v amdgpu | tee -a $O/budget.txt || exit 1
timeout -k 10 300 python -u tools/f64_budget.py c2 500 40 96 2>&1 | grep -v amdgpu | tee -a $O/budget.txt || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_blobs.py::test_float64_input_identical_to_reference "tests/test_gpu_api.py::test_corr_csv_configs" tests/test_gpu_api.py::test_auto_precision_float64_input_is_f64 "tests/test_gpu_kmeans.py::test_f64_labels_match_sklearn_float64" "tests/test_gpu_kmeans.py::test_f64_relocation_with_ties_is_pinned" -q --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
