# float64 k-means (cc_kmeans_f64) rework: bit-identity against the previous kernel
# (libccmi_f64_base.so) at the C2 and C3 shapes, the float64 parity tests, and timings.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4f; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_blobs.py::test_float64_input_identical_to_reference "tests/test_gpu_api.py::test_corr_csv_configs" tests/test_gpu_api.py::test_auto_precision_float64_input_is_f64 "tests/test_gpu_kmeans.py::test_f64_labels_match_sklearn_float64" "tests/test_gpu_kmeans.py::test_f64_relocation_with_ties_is_pinned" -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|float64 input|f64 relocation" $O/tests.log | tail -10; [ $rc -eq 0 ] || exit $rc
for c in "c2 16" "c3 8"; do
  set -- $c
  timeout -k 10 300 python -u tools/f64_ab.py $1 $2 /tmp/new_$1.npz 2>&1 | grep -v amdgpu || exit 1
  CCMI_LIB=consensus_clustering_amd/libccmi_f64_base.so timeout -k 10 300 python -u tools/f64_ab.py $1 $2 /tmp/base_$1.npz 2>&1 | grep -v amdgpu || exit 1
  python tools/f64_ab.py --compare /tmp/new_$1.npz /tmp/base_$1.npz || exit 1
done
timeout -k 10 600 python -u tools/gmm_time.py 10000 16 32 > $O/gmm_time.txt 2>&1; grep -v amdgpu $O/gmm_time.txt
# k-means compiler-scheduling variants (tools/build_variant.sh flags), C3 launch alone
LIBS="libccmi_kv_base.so libccmi_kv_ptr.so libccmi_kv_trk.so libccmi_kv_nohrp.so libccmi_kv_bias0.so libccmi_kv_bias100.so libccmi_kv_noclo.so libccmi_kv_noDE.so libccmi_kv_base.so" KM_H=1000 KM_CFG=c3 bash tools/gpu_ab.sh 2>&1 | grep -v amdgpu | tee $O/kv_ab.txt
for c in c3 c2; do timeout -k 10 120 python -u tools/rs_time.py $c 3 2>&1 | grep -v amdgpu | tee -a $O/rs_time.txt; done
