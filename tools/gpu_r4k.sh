# k-means variant A/B (labels by digest, HIP-event launch time) at C3 / C5 / C2, full grid.
set -o pipefail
export TMPDIR=/tmp KM_BUDGET_GB=40
O=$GRAFT_REPO_ROOT/gpurun_out/r4k; mkdir -p $O
cd $GRAFT_REPO_ROOT
for cfg in "c3 1000" "c5 256" "c2 500"; do
  set -- $cfg
  LIBS="${KV_LIBS:-libccmi_kv_base.so libccmi_kv_amin.so libccmi_kv_base.so libccmi_kv_amin.so}" KM_H=$2 KM_CFG=$1 bash tools/gpu_ab.sh 2>&1 | grep -v amdgpu | grep -v "sweeps by active" | tee -a $O/kv_ab.txt || exit 1
done
