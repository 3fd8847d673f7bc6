# k-means launch alone (HIP events, 40 GB budget) for library variants at several configs:
# times and label / inertia / n_iter digests.  VARS="prev img" CFGS="c3:1000 c5:256 c2:500"
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f; mkdir -p $O
export KM_BUDGET_GB=40
for c in ${CFGS:-c3:1000}; do
  cfg=${c%%:*}; H=${c##*:}
  for v in ${VARS:-prev}; do
    CCMI_LIB=$PWD/consensus_clustering_amd/libccmi_$v.so timeout -k 10 300 python -u tools/km_time.py $H $cfg ${REPS:-2} > $O/km_${cfg}_$v.txt 2>&1 || { echo FAIL $v $cfg; tail -5 $O/km_${cfg}_$v.txt; exit 1; }
    echo "$cfg $(grep -v amdgpu.ids $O/km_${cfg}_$v.txt | head -1)"
  done
done
