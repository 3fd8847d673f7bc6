# rocprofv3 kernel-trace summary of the C4 fit (the wide engine's E / M / P split).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4s; mkdir -p $O
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o c4 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof.log; exit 1; }
head -12 $O/prof/c4_kernel_stats.csv | cut -c1-160
