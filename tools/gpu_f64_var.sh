# A/B of a float64 k-means variant library against libccmi_f64_base.so (identity + time):
#   bash tools/gpu_f64_var.sh NAME   (consensus_clustering_amd/libccmi_NAME.so)
set -o pipefail
export TMPDIR=/tmp
V=$1
O=$GRAFT_REPO_ROOT/gpurun_out/f64var_$V; mkdir -p $O
cd $GRAFT_REPO_ROOT
for c in ${F64_CFGS:-c2:16 c3:8 c2:128}; do
  set -- ${c/:/ }
  CCMI_LIB=consensus_clustering_amd/libccmi_$V.so timeout -k 10 300 python -u tools/f64_ab.py $1 $2 /tmp/new_$1.npz 2>&1 | grep -v amdgpu || exit 1
  CCMI_LIB=consensus_clustering_amd/libccmi_f64_base.so timeout -k 10 300 python -u tools/f64_ab.py $1 $2 /tmp/base_$1.npz 2>&1 | grep -v amdgpu || exit 1
  python tools/f64_ab.py --compare /tmp/new_$1.npz /tmp/base_$1.npz | tee -a $O/ab.txt || exit 1
done
