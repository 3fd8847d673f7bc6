"""Summarise tools/gpu_pmc.sh output for the k-means kernel (per wave and tile iteration)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = collections.defaultdict(float)
for f in sorted(glob.glob(f"{root}/p*/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "kmeans" in r["Kernel_Name"] and "_kernel" in r["Kernel_Name"] and "split" not in r["Kernel_Name"]:
            vals[r["Counter_Name"]] += float(r["Counter_Value"])
st = eval(open(f"{root}/p1.log").read().split("stats")[1].strip().splitlines()[0])
w = vals["SQ_WAVES"]
iters = st[4] * 1252 / (w / 8)
print("iterations per wave %.0f, active slot tiles per iteration %.2f" % (iters, st[5] / (st[4] * 1250)))
print("per wave-iteration: " + " ".join("%s %.1f" % (k.replace("SQ_INSTS_", ""), vals[k] / w / iters)
                                        for k in ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA",
                                                  "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH"]))
tot = vals["SQ_WAVE_CYCLES"]
print("wave-cycle split: wait_any %.0f%% wait_inst %.0f%% active %.0f%%" % (
    100 * vals["SQ_WAIT_ANY"] / tot, 100 * vals["SQ_WAIT_INST_ANY"] / tot, 100 * vals["SQ_ACTIVE_INST_ANY"] / tot))
print("LDS bank conflict / active: %.2f" % (vals["SQ_LDS_BANK_CONFLICT"] / max(vals["SQ_LDS_IDX_ACTIVE"], 1)))
print("MFMA busy / busy cycles: %.2f, coexec / mfma busy %.2f" % (
    vals["SQ_VALU_MFMA_BUSY_CYCLES"] / max(vals["SQ_BUSY_CYCLES"], 1) / 4,
    vals["SQ_VALU_MFMA_COEXEC_CYCLES"] / max(vals["SQ_VALU_MFMA_BUSY_CYCLES"], 1)))
