# co-association timing (C3) for the default library and the build variants named in VARS
export TMPDIR=/tmp
for v in "" $VARS; do
  if [ -z "$v" ]; then lib=consensus_clustering_amd/libccmi.so; else lib=consensus_clustering_amd/libccmi_$v.so; fi
  echo "== ${v:-default}"
  CCMI_LIB=$lib timeout -k 10 200 python -u tools/co_only.py ${CFG:-c3} 2>&1 | grep -v amdgpu | tail -2 || exit 1
done
