"""Per-kernel register / scratch / LDS usage of a HIP source for gfx950, from the compiler's
-Rpass-analysis=kernel-resource-usage remarks (demangled kernel names, one line per kernel).

    python tools/resource_usage.py consensus_clustering_amd/csrc/kmeans.hip [extra hipcc flags]
"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-function",
       "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?):\s+(.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        dm = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()
        cur = {"kernel": dm.replace("(anonymous namespace)::", "")}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
cols = ["VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
print("kernel | " + " | ".join(cols))
for r in rows:
    print(r["kernel"][:90], "|", " | ".join(r.get(c, "-") for c in cols))
