# float64 multi-K units: A/B (identity + time) of libccmi_${V:-kp2}.so against libccmi_f64_base.so at
# two K's per unit (default) and one (CCMI_F64_KPACK=1), then the f64 GPU tests on the variant.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5l; mkdir -p $O
F64_CFGS="c3:128 c2:500" bash tools/gpu_f64_var.sh ${V:-kp2} > $O/ab_p2.txt 2>&1 || { cat $O/ab_p2.txt; exit 1; }
cat $O/ab_p2.txt
CCMI_F64_KPACK=1 F64_CFGS="c3:128" bash tools/gpu_f64_var.sh ${V:-kp2} > $O/ab_p1.txt 2>&1 || { cat $O/ab_p1.txt; exit 1; }
cat $O/ab_p1.txt
CCMI_LIB=consensus_clustering_amd/libccmi_${V:-kp2}.so timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -k "f64 or float64" \
  tests/test_gpu_kmeans.py tests/test_gpu_parity_blobs.py tests/test_gpu_api.py tests/test_gpu_fit.py > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -20
exit $rc
