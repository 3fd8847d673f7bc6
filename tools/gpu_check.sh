#!/bin/bash
# GPU tests, then (unless the tests hit a fault/timeout) a short C3 bench with the CPU baseline.
# Usage (from the repo root, on the GPU box): bash tools/gpu_check.sh [pytest -k expr]
OUT=gpurun_out
mkdir -p $OUT
K=${1:+-k "$1"}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread --maxfail=6 $K > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -25 $OUT/tests.log
case $rc in 124|137|134|139) echo "fault/timeout: stopping"; exit $rc;; esac
if [ -n "$NOBENCH" ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err
brc=$?
echo "bench rc=$brc"; cat $OUT/bench.json; tail -5 $OUT/bench.err
exit $rc
