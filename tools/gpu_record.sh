# Full GPU check + bench (with CPU baseline) + rocprofv3 kernel-trace summary of the bench.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/rec
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; echo "TESTS rc=$?"; grep -cE "PASSED" $OUT/gpu_tests.log; grep -E "FAILED|ERROR" $OUT/gpu_tests.log | head
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -5 $OUT/bench.err; exit 1; }
echo BENCH_OK
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c3 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo PROF_FAIL; tail -5 $OUT/prof.log; exit 1; }
echo PROF_OK
