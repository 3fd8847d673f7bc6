# float64 multi-K units: base once per config, then the variant under several grouping settings
# (SETTINGS: library:CCMI_F64_KPACK:CCMI_F64_KPAIR_MAX ...), each compared with the base (identity + time).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
V=${V:-kp4}
O=gpurun_out/r5n; mkdir -p $O
for c in ${F64_CFGS:-c3:128 c2:500}; do
  set -- ${c/:/ }
  CCMI_LIB=consensus_clustering_amd/libccmi_f64_base.so timeout -k 10 300 python -u tools/f64_ab.py $1 $2 /tmp/base_$1.npz 2>&1 | grep -v amdgpu || exit 1
  for s in ${SETTINGS:-$V:1:127 $V:2:127}; do
    set -- ${c/:/ } ${s//:/ }
    if [ "$4" = auto ]; then unset CCMI_F64_KPACK; else export CCMI_F64_KPACK=$4; fi
    CCMI_F64_KPAIR_MAX=$5 CCMI_LIB=consensus_clustering_amd/libccmi_$3.so timeout -k 10 300 python -u tools/f64_ab.py $1 $2 /tmp/new_$1.npz 2>&1 | grep -v amdgpu || exit 1
    echo -n "$3 P=$4 Kpair<=$5: " | tee -a $O/ab.txt
    python tools/f64_ab.py --compare /tmp/new_$1.npz /tmp/base_$1.npz | tee -a $O/ab.txt || exit 1
  done
done
