"""Summarise tools/gpu_sq.sh passes for the dispatches whose kernel name contains FILTER.

    python tools/sq_summary.py <dir> <filter>      (filter: "a,b,-c" = contains a and b, not c)

Units (MI355X_MICROARCH.md, 'rocprofv3 PMC slots' and the cycle-constant rows):
- SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles, summed over waves;
- SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles with the matrix pipe busy, summed over SIMDs
  (32 per v_mfma_*_32x32x16_f16 / 32x32x32_i8);
- GRBM_GUI_ACTIVE is the GPU-busy cycle count summed over the 8 XCDs, so one XCD's (= the
  chip's) elapsed cycles are GRBM_GUI_ACTIVE / 8.
MFMA busy % = SQ_VALU_MFMA_BUSY_CYCLES / (elapsed cycles x 256 CUs x 4 SIMDs).
"""
import collections
import csv
import glob
import sys

N_SIMD = 256 * 4

root, filt = sys.argv[1], sys.argv[2]
inc = [t for t in filt.split(",") if t and not t.startswith("-")]
exc = [t[1:] for t in filt.split(",") if t.startswith("-")]


def wanted(name):
    return all(t in name for t in inc) and not any(t in name for t in exc)


per_pass = []
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    v = collections.defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(f)):
        if wanted(r["Kernel_Name"]):
            v[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    per_pass.append((f, v, len(disp)))
vals = collections.defaultdict(float)
for _, v, _ in per_pass:
    for k, x in v.items():
        if k != "GRBM_GUI_ACTIVE":
            vals[k] += x
grbm = [v["GRBM_GUI_ACTIVE"] for _, v, _ in per_pass if v.get("GRBM_GUI_ACTIVE")]
ndisp = [nd for _, _, nd in per_pass]
w = max(vals["SQ_WAVES"], 1)
tot = max(vals["SQ_WAVE_CYCLES"], 1)
elapsed = grbm[1] / 8 if len(grbm) > 1 else (grbm[0] / 8 if grbm else 0)  # pass 2 holds MFMA busy
print(f"filter '{filt}': dispatches per pass {ndisp}, waves {w:.0f}")
print("per wave: " + " ".join("%s %.0f" % (k.replace("SQ_INSTS_", ""), vals[k] / w) for k in
                              ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA",
                               "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH"]))
print("VALU / MFMA instructions: %.2f" % (vals["SQ_INSTS_VALU"] / max(vals["SQ_INSTS_MFMA"], 1)))
print("wave-cycle split: wait_any (s_waitcnt/barrier) %.1f%%, wait_inst (issue stall) %.1f%%, active %.1f%%"
      % (100 * vals["SQ_WAIT_ANY"] / tot, 100 * vals["SQ_WAIT_INST_ANY"] / tot, 100 * vals["SQ_ACTIVE_INST_ANY"] / tot))
print("LDS bank conflict cycles / LDS active cycles: %.3f" % (vals["SQ_LDS_BANK_CONFLICT"] / max(vals["SQ_LDS_IDX_ACTIVE"], 1)))
if elapsed:
    busy = vals["SQ_VALU_MFMA_BUSY_CYCLES"]
    print("elapsed %.4g cycles per pass (GRBM_GUI_ACTIVE/8, summed over the filtered dispatches)" % elapsed)
    print("MFMA busy: %.1f%% of SIMD cycles (SQ_VALU_MFMA_BUSY_CYCLES %.4g / (%.4g x %d SIMDs))"
          % (100 * busy / (elapsed * N_SIMD), busy, elapsed, N_SIMD))
    print("MFMA busy cycles per MFMA instruction: %.1f" % (busy / max(vals["SQ_INSTS_MFMA"], 1)))
    print("VALU+MFMA co-issue / MFMA busy: %.2f" % (vals["SQ_VALU_MFMA_COEXEC_CYCLES"] / max(busy, 1)))
