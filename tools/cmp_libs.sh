set -o pipefail
mkdir -p gpurun_out/cmp
for lib in ${LIBS:-libccmi_prev.so libccmi.so}; do
  for c in c5 c2; do
    CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/$lib timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cmp/$lib.$c.json 2>/dev/null || { echo FAIL $lib $c; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/cmp/$lib.$c.json').read().strip().splitlines()[-1]);print('$lib $c', d['kernels_ms_per_step'])"
  done
done
