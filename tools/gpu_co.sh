# Co-association kernel: per-K timings at C3 shape, then PMC passes for one K (CO_K, default 20).
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/co
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/co_only.py ${CO_CFG:-c3} > $OUT/t.txt 2>&1 || { echo FAIL; tail -3 $OUT/t.txt; exit 1; }
grep -v amdgpu.ids $OUT/t.txt
[ -n "${CO_PMC:-}" ] || exit 0
cd /tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o p$i --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/co_only.py ${CO_CFG:-c3} ${CO_K:-20} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import collections, csv, glob, os
root = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/co"
v = collections.defaultdict(float)
for f in glob.glob(root + "/p*/p*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "tiles_kernel" in r["Kernel_Name"] and "<1>" not in r["Kernel_Name"]:
            v[r["Counter_Name"]] += float(r["Counter_Value"])
w = v["SQ_WAVES"]
print({k: round(x / w) for k, x in sorted(v.items())})
tot = v["SQ_WAVE_CYCLES"]
print("wait_any %.2f wait_inst %.2f active %.2f valu %.2f lds %.2f" % tuple(v[k] / tot for k in ["SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"]))
print("mfma busy/busy %.2f coexec/mfma %.2f lds conflict/active %.3f" % (v["SQ_VALU_MFMA_BUSY_CYCLES"] / max(v["SQ_BUSY_CYCLES"], 1) / 4, v["SQ_VALU_MFMA_COEXEC_CYCLES"] / max(v["SQ_VALU_MFMA_BUSY_CYCLES"], 1), v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_LDS_IDX_ACTIVE"], 1)))
PY
