# float64 k-means with the tiled E-step: the float64 parity tests, then bit-identity and timing
# against the previous kernel (libccmi_f64_base.so) at the C2 and C3 shapes.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4ad; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_blobs.py::test_float64_input_identical_to_reference "tests/test_gpu_api.py::test_corr_csv_configs" tests/test_gpu_api.py::test_auto_precision_float64_input_is_f64 "tests/test_gpu_kmeans.py::test_f64_labels_match_sklearn_float64" "tests/test_gpu_kmeans.py::test_f64_relocation_with_ties_is_pinned" -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|float64 input|f64 relocation" $O/tests.log | tail -10; [ $rc -eq 0 ] || exit $rc
for c in "c2 16" "c3 8" "c2 128"; do
  set -- $c
  timeout -k 10 300 python -u tools/f64_ab.py $1 $2 /tmp/new_$1.npz 2>&1 | grep -v amdgpu || exit 1
  CCMI_LIB=consensus_clustering_amd/libccmi_f64_base.so timeout -k 10 300 python -u tools/f64_ab.py $1 $2 /tmp/base_$1.npz 2>&1 | grep -v amdgpu || exit 1
  python tools/f64_ab.py --compare /tmp/new_$1.npz /tmp/base_$1.npz | tee -a $O/ab.txt || exit 1
done
