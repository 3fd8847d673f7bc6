# Build a variant library from an alternative kmeans.hip (A/B runs through CCMI_LIB):
#   bash tools/build_variant.sh NAME path/to/kmeans_variant.hip [extra HIPFLAGS]
# -> consensus_clustering_amd/libccmi_NAME.so.  Builds in a private copy of the sources
# (/tmp/ccmi_variant_NAME/consensus_clustering_amd/csrc), so variants can build in parallel.
set -e
NAME=$1; SRC=$(readlink -f "$2"); shift 2
REPO=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/ccmi_variant_$NAME
rm -rf $W && mkdir -p $W/consensus_clustering_amd $W/include
cp -r $REPO/consensus_clustering_amd/csrc $W/consensus_clustering_amd/
cp $REPO/include/ccmi.h $W/include/
cp "$SRC" $W/consensus_clustering_amd/csrc/kmeans.hip
[ -n "$CO_SRC" ] && cp "$CO_SRC" $W/consensus_clustering_amd/csrc/coassoc.hip  # a coassoc.hip variant (with REBUILD=coassoc)
[ -n "$PR_SRC" ] && cp "$PR_SRC" $W/consensus_clustering_amd/csrc/predict.hip  # a predict.hip variant (with REBUILD=predict)
[ -n "$F64_SRC" ] && cp "$F64_SRC" $W/consensus_clustering_amd/csrc/kmeans_f64.hip  # a kmeans_f64.hip variant (with REBUILD=kmeans_f64)
[ -n "$WIDE_SRC" ] && cp "$WIDE_SRC" $W/consensus_clustering_amd/csrc/kmeans_wide.hip  # a kmeans_wide.hip variant (with REBUILD=kmeans_wide)
mkdir -p $W/build
cp $REPO/build/ccmi/*.o $W/build/ 2>/dev/null || true  # unchanged objects are reused (kmeans.o rebuilds)
for o in kmeans $REBUILD; do rm -f $W/build/$o.o; done  # REBUILD="coassoc ...": objects whose flags change
touch $W/build/*.o 2>/dev/null || true
cd $W/consensus_clustering_amd/csrc
make -j4 HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -falign-loops=64 $*" \
  OUT=$REPO/consensus_clustering_amd/libccmi_$NAME.so BUILD=$W/build > $W/build.log 2>&1 || { tail -20 $W/build.log; exit 1; }
echo built libccmi_$NAME.so
