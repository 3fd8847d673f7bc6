# SQ counter passes (plus GRBM_GUI_ACTIVE for the clock) on one driver, summarised per kernel
# by tools/sq_summary.py: MFMA busy as a % of SIMD cycles, VALU/MFMA, wait split, LDS conflicts.
#   SQ_TAG=km_c3 SQ_FILTER=kmeans_kernel bash tools/gpu_sq.sh tools/km_only.py 1000 c3
#   SQ_TAG=co_c3 SQ_FILTER=tiles_kernel  bash tools/gpu_sq.sh tools/co_only.py c3
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/sq_${SQ_TAG:-run}
mkdir -p $OUT
# the driver script path is taken relative to the repository root
SCRIPT=$1; shift
case "$SCRIPT" in /*) ;; *) SCRIPT=$GRAFT_REPO_ROOT/$SCRIPT ;; esac
cd /tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d $OUT/p$i -o p$i --output-format csv -- python3 "$SCRIPT" "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/sq_summary.py $OUT "${SQ_FILTER:-kernel}" | tee $OUT/summary.txt
