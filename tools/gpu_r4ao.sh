# rocprofv3 kernel trace of the float64 engine at the C3 shape (H = 32) and C2 (H = 128)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r4ao; mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o f64_c3 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/f64_time.py c3 32 > $O/prof_c3.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_c3.log; exit 1; }
grep -v amdgpu $O/prof_c3.log | tail -3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o f64_c2 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/f64_time.py c2 128 > $O/prof_c2.log 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_c2.log; exit 1; }
grep -v amdgpu $O/prof_c2.log | tail -3
