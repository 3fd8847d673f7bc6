# Determinism of float64 k-means builds: each library run twice per config, results compared.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for v in ${VARS:-f64_base f64mg8}; do
  for c in ${F64_CFGS:-c2:500}; do
    set -- ${c/:/ }
    for rep in 1 2 3; do
      CCMI_LIB=consensus_clustering_amd/libccmi_$v.so timeout -k 10 300 python -u tools/f64_ab.py $1 $2 /tmp/${v}_$1_$rep.npz 2>&1 | grep -v amdgpu || exit 1
    done
    echo "$v $c run1 vs run2: $(python tools/f64_ab.py --compare /tmp/${v}_$1_1.npz /tmp/${v}_$1_2.npz)"
    echo "$v $c run1 vs run3: $(python tools/f64_ab.py --compare /tmp/${v}_$1_1.npz /tmp/${v}_$1_3.npz)"
  done
done
