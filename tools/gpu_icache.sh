# Instruction-cache counters of the k-means launch for library variants (ICACHE_LIBS), H=256.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/icache; mkdir -p $O
cd /tmp
for lib in $ICACHE_LIBS; do
  export CCMI_LIB=$GRAFT_REPO_ROOT/consensus_clustering_amd/$lib
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE -d $O/$lib -o ic --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/km_only.py 256 c3 > $O/$lib.log 2>&1 || { echo "pass failed $lib"; tail -5 $O/$lib.log; exit 1; }
  python3 - "$O/$lib" "$lib" <<'PY'
import csv, glob, sys, collections
d, lib = sys.argv[1], sys.argv[2]
f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
tot = collections.defaultdict(float)
for fn in f:
    for r in csv.DictReader(open(fn)):
        if "kmeans_kernel" in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
h, m = tot["SQC_ICACHE_HITS"], tot["SQC_ICACHE_MISSES"]
print(lib, {k: f"{v:.3e}" for k, v in tot.items()}, "miss rate %.4f" % (m / max(h + m, 1)))
PY
done
