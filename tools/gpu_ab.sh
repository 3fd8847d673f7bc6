# A/B of the k-means launch alone (HIP events) for several library builds at one config:
# LIBS="libccmi_prev.so libccmi.so" KM_H=1000 KM_CFG=c3 bash tools/gpu_ab.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/ab
cd $GRAFT_REPO_ROOT
for lib in ${LIBS:-libccmi_prev.so libccmi.so}; do
  CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/$lib timeout -k 10 300 python -u tools/km_time.py ${KM_H:-1000} ${KM_CFG:-c3} ${KM_REPS:-2} || { echo FAIL $lib; exit 1; }
done
