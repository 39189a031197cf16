"""Per-kernel medians of the tools/pmc_step.sh passes (one dispatch = one launch of the kernel in a
bench step): HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, the gfx950 FETCH_SIZE correction of
MI355X_MICROARCH.md), MFMA busy cycles and op counts.  python3 tools/pmc_step_summary.py DIR"""
import collections
import csv
import glob
import json
import statistics
import sys

KERNELS = ("march_train_walk2", "march_train_place", "field_fwd_kernel", "field_bwd_kernel", "field_scatter_kernel",
           "composite_fw_kernel", "composite_bw_kernel", "cluster_kernel", "adam_prep", "adam_apply")
d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(dict))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
        if k is None:
            continue
        if k == "field_bwd_kernel":  # the split backward's passes (template PART 1 / 2; 3 = one pass)
            part = next((p for p in ("1", "2", "3") if f"Li{p}E" in r["Kernel_Name"]), "3")
            k += {"1": " (rgb pass)", "2": " (sigma pass)", "3": " (one pass)"}[part]
        key = (f, r["Dispatch_Id"])
        vals[k][r["Counter_Name"]][key] = vals[k][r["Counter_Name"]].get(key, 0.0) + float(r["Counter_Value"])
out = {}
for k, cs in vals.items():
    med = {c: statistics.median(v.values()) for c, v in cs.items()}
    e = {"counters_median_per_dispatch": med, "dispatches": {c: len(v) for c, v in cs.items()}}
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:  # KB units
        e["hbm_bytes_per_launch"] = (2 * med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024
    out[k] = e
print(json.dumps(out, indent=1))
