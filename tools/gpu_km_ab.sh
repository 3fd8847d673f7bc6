# k-means launch alone (HIP events) at the configs in KM_CFGS for each library in KM_LIBS
# (default: the in-tree libccmi.so):  KM_LIBS="libccmi_prev.so libccmi.so" bash tools/gpu_km_ab.sh
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/kmab; mkdir -p $O
for cfg in ${KM_CFGS:-c3 c5 c2}; do
  case $cfg in c3) H=1000;; c5) H=256;; c2) H=500;; *) H=${KM_H:-256};; esac
  for lib in ${KM_LIBS:-libccmi.so}; do
    CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/$lib timeout -k 10 200 python -u tools/km_time.py $H $cfg 2 > $O/km_${cfg}_$lib.txt 2>&1 || { echo km $lib $cfg fail; tail -3 $O/km_${cfg}_$lib.txt; exit 1; }
    echo "== $cfg $lib: $(grep 'kmeans ms' $O/km_${cfg}_$lib.txt)"
  done
done
