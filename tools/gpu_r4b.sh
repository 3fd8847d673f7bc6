# Full GPU suite after the round-4 parity changes (sk_parity without the fixed-point clause, the
# single-path exchange in dist.py, the hybrid path over n_jobs).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4b; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed|sklearn parity|FAILED" $O/gpu_tests.log | tail -30; exit $rc
