# TCP probe: the f64 E-step with contiguous 512-B B-operand loads (wrong values, same work) -
# per-iteration E-step cost against the stamps build of HEAD
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4ag; mkdir -p $O
cd $GRAFT_REPO_ROOT
CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/libccmi_f64tcp.so timeout -k 10 300 python -u tools/f64_stamps.py c3 8 c2 128 2>&1 | grep -v amdgpu | tee $O/stamps_tcp.txt || exit 1
