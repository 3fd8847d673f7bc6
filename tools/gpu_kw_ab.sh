# Wide-engine A/B: the default library against LIB_B (consensus_clustering_amd/libccmi_<name>.so) on
# C4-shaped expression data (tools/wide_labels_dump.py n d H), labels / inertia / n_iter compared.
#   LIB_B=libccmi_wbase.so KW_SHAPE="5000 20000 1000" bash tools/gpu_kw_ab.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/kw
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/wide_labels_dump.py gpurun_out/kw/a.npz ${KW_SHAPE:-5000 20000 1000} 2>&1 | grep -v amdgpu.ids || exit 1
CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/${LIB_B:-libccmi_wbase.so} timeout -k 10 300 python -u tools/wide_labels_dump.py gpurun_out/kw/b.npz ${KW_SHAPE:-5000 20000 1000} 2>&1 | grep -v amdgpu.ids || exit 1
python -c "
import numpy as np
a=np.load('gpurun_out/kw/a.npz'); b=np.load('gpurun_out/kw/b.npz')
print('labels equal', np.array_equal(a['L'],b['L']), 'inertia equal', np.array_equal(a['inert'],b['inert']), 'n_iter equal', np.array_equal(a['nit'],b['nit']))
"
rm -f gpurun_out/kw/*.npz
