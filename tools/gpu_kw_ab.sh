export TMPDIR=/tmp
mkdir -p gpurun_out/kw
timeout -k 10 300 python -u tools/wide_labels_dump.py gpurun_out/kw/a.npz 5000 20000 1000 2>&1 | grep -v amdgpu.ids || exit 1
CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/libccmi_kwnoalign.so timeout -k 10 300 python -u tools/wide_labels_dump.py gpurun_out/kw/b.npz 5000 20000 1000 2>&1 | grep -v amdgpu.ids || exit 1
python -c "
import numpy as np
a=np.load('gpurun_out/kw/a.npz'); b=np.load('gpurun_out/kw/b.npz')
print('labels equal', np.array_equal(a['L'],b['L']), 'inertia equal', np.array_equal(a['inert'],b['inert']), 'n_iter equal', np.array_equal(a['nit'],b['nit']))
"
rm -f gpurun_out/kw/*.npz
