# r02 profiles: rocprofv3 kernel stats of a C3 bench run, then FETCH_SIZE / WRITE_SIZE passes (one
# counter group per run, as the MI355X guide prescribes) over one C3 fit; summarised into
# profiles/traffic/ by tools/traffic_summary.py (run on the host afterwards).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof
mkdir -p $OUT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o c3 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/stats.log 2>&1 || { echo "stats pass failed"; tail -5 $OUT/stats.log; exit 1; }
tail -1 $OUT/stats.log
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d $OUT/$C -o $C --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/$C.log 2>&1 || { echo "$C pass failed"; tail -5 $OUT/$C.log; exit 1; }
done
echo TRAFFIC_OK
