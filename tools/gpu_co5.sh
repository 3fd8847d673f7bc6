# co-association: per-K timings of the HEAD library and of variants (CO_VARIANTS), per config
# (CO_CFGS, default c5), then phase stamps of the diagnostic build libccmi_costamps.so
export TMPDIR=/tmp
mkdir -p gpurun_out/co5
for c in ${CO_CFGS:-c5}; do
  timeout -k 10 200 python -u tools/co_only.py $c > gpurun_out/co5/$c.txt 2>&1 || exit $?
  echo "== $c HEAD"; grep -v amdgpu.ids gpurun_out/co5/$c.txt | tail -2
  for v in ${CO_VARIANTS:-}; do
    CCMI_LIB=consensus_clustering_amd/libccmi_$v.so timeout -k 10 200 python -u tools/co_only.py $c > gpurun_out/co5/${c}_$v.txt 2>&1 || exit $?
    echo "== $c $v"; grep -v amdgpu.ids gpurun_out/co5/${c}_$v.txt | tail -2
  done
done
CCMI_LIB=consensus_clustering_amd/libccmi_costamps.so timeout -k 10 200 python -u tools/co_stamps.py c5 ${CO_KS:-2 5 9} > gpurun_out/co5/stamps.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/co5/stamps.txt
