# k-means pair mode (two row tiles per barrier in narrow sweeps, d <= 64): label digests and
# launch times against the base build at C5 / C2, and the C3 launch (d = 128 must be unchanged).
set -o pipefail
export TMPDIR=/tmp KM_BUDGET_GB=40
O=$GRAFT_REPO_ROOT/gpurun_out/r4y; mkdir -p $O
cd $GRAFT_REPO_ROOT
for cfg in "c5 256" "c2 500"; do
  set -- $cfg
  LIBS="libccmi_kv_base.so libccmi_kv_pcs.so libccmi_kv_pcs2.so libccmi_kv_base.so libccmi_kv_pcs.so libccmi_kv_pcs2.so" KM_H=$2 KM_CFG=$1 bash tools/gpu_ab.sh 2>&1 | grep -v amdgpu | grep -v "sweeps by active" | tee -a $O/kv_ab.txt || exit 1
done
LIBS="libccmi_kv_base.so libccmi_kv_pcs2.so libccmi_kv_pcs.so" KM_H=1000 KM_CFG=c3 bash tools/gpu_ab.sh 2>&1 | grep -v amdgpu | grep -v "sweeps by active" | tee -a $O/kv_ab.txt
