# Sparse vs dense M-step diagnostics on C3-shaped blobs (two data seeds), then the C3 k-means
# launch with the CCMI_KM_DENSE switch compiled in (kv_dflag) against the build without it.
set -o pipefail
export TMPDIR=/tmp KM_BUDGET_GB=40
O=$GRAFT_REPO_ROOT/gpurun_out/r4m; mkdir -p $O
cd $GRAFT_REPO_ROOT
for s in 11 5; do timeout -k 10 400 python -u tools/sparse_dense_diag.py 4000 $s 4 2>&1 | grep -v amdgpu | tee -a $O/diag.txt || exit 1; done
LIBS="libccmi_kv_base.so libccmi_kv_dflag.so libccmi_kv_base.so libccmi_kv_dflag.so" KM_H=1000 KM_CFG=c3 bash tools/gpu_ab.sh 2>&1 | grep -v amdgpu | grep -v "sweeps by active" | tee $O/kv_ab.txt
