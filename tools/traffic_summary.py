"""Summarise tools/gpu_traffic.sh output into profiles/traffic/<config>_<kernel>.json.

    python tools/traffic_summary.py gpurun_out/prof c3 r02

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  Per MI355X_MICROARCH.md (HBM section),
FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads on gfx950, so it is doubled;
WRITE_SIZE is taken as is.  Both count L2 -> fabric traffic (Infinity-Cache hits included).
"""
import collections
import csv
import glob
import json
import os
import sys

root, config, tag = sys.argv[1], sys.argv[2], sys.argv[3]
# tiles_kernel<1, false> is the co-sampling instantiation (demangled names carry every template
# argument)
KERNELS = {"cc_kmeans_batched": lambda k: "kmeans_kernel" in k,
           "cc_coassoc": lambda k: "tiles_kernel" in k and "tiles_kernel<1," not in k,
           "cc_cosample": lambda k: "tiles_kernel<1," in k}
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{root}/{ctr}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != ctr:
                continue
            for name, match in KERNELS.items():
                if match(r["Kernel_Name"]):
                    tot[(name, ctr)] += float(r["Counter_Value"])
                    disp[(name, ctr)].add(r.get("Dispatch_Id", r.get("Correlation_Id", len(disp[(name, ctr)]))))
os.makedirs("profiles/traffic", exist_ok=True)
for name in KERNELS:
    n = len(disp[(name, "FETCH_SIZE")])
    if n == 0:
        continue
    rd = 2.0 * tot[(name, "FETCH_SIZE")] * 1024
    wr = tot[(name, "WRITE_SIZE")] * 1024
    out = {"kernel": name, "workload": f"{config} full fit (bench.py --config {config} --steps 1 --warmup 0)",
           "dispatches_per_fit": n, "read_bytes_per_fit": rd, "write_bytes_per_fit": wr,
           "bytes_per_fit": rd + wr, "bytes_per_launch": (rd + wr) / n,
           "correction": "FETCH_SIZE (KiB) doubled (gfx950: half the bytes of 16-B-per-lane streaming reads), "
                         "WRITE_SIZE (KiB) as is; L2 -> fabric traffic, Infinity-Cache hits included",
           "source": f"profiles/pmc/{tag}_{config}_fetch_size.csv, profiles/pmc/{tag}_{config}_write_size.csv "
                     "(separate --pmc runs)"}
    json.dump(out, open(f"profiles/traffic/{config}_{name}.json", "w"), indent=1)
    print(name, {k: (f"{v / 1e9:.2f} GB" if isinstance(v, float) and v > 1e6 else v) for k, v in out.items()
                 if k.endswith(("fit", "launch"))})
