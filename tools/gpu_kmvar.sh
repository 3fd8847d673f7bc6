# k-means launch time (C3 shape) for the default library and the build variants named in VARS
export TMPDIR=/tmp
for v in "" $VARS; do
  if [ -z "$v" ]; then lib=consensus_clustering_amd/libccmi.so; else lib=consensus_clustering_amd/libccmi_$v.so; fi
  CCMI_LIB=$lib timeout -k 10 200 python -u tools/km_time.py ${H:-1000} c3 2 2>&1 | grep -v amdgpu || exit 1
done
