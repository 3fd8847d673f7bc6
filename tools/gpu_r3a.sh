# Round 3 first GPU pass: HEAD k-means SQ counters; FP4 co-association tests and timings
# (default packing, forced power-of-two packing, the round-2 i8 library), co-association SQ.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3a
SQ_TAG=km_c3 SQ_FILTER=kmeans_kernel timeout -k 10 500 bash tools/gpu_sq.sh tools/km_only.py 1000 c3 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_coassoc.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3a/co_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3a/co_tests.log; [ $rc -eq 0 ] || exit $rc
for v in default pow2 r02; do
  case $v in
    default) timeout -k 10 200 python -u tools/co_only.py c3 > gpurun_out/r3a/co_$v.txt 2>&1 ;;
    pow2) CCMI_CO_PACK=pow2 timeout -k 10 200 python -u tools/co_only.py c3 > gpurun_out/r3a/co_$v.txt 2>&1 ;;
    r02) CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/libccmi_r02co.so timeout -k 10 200 python -u tools/co_only.py c3 > gpurun_out/r3a/co_$v.txt 2>&1 ;;
  esac || { echo "co_only $v failed"; tail -3 gpurun_out/r3a/co_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/r3a/co_$v.txt
done
timeout -k 10 200 python -u tools/co_only.py c5 > gpurun_out/r3a/co_c5.txt 2>&1 && grep -v amdgpu.ids gpurun_out/r3a/co_c5.txt
SQ_TAG=co_c3 SQ_FILTER=tiles_kernel,-"<1," timeout -k 10 400 bash tools/gpu_sq.sh tools/co_only.py c3
