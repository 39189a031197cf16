"""Summarise tools/pmc_calib.sh (gpurun_out/pmc_calib): per kernel, the median per-dispatch
FETCH_SIZE and WRITE_SIZE (KB counters x 1024) against the bytes the kernel moves."""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "pmc_calib")
KNOWN = {"k_stream16": 256 << 20, "k_chunk48": 256 << 20, "k_chunk24": 256 << 20, "k_pair8": 256 << 20,
         "k_atomics": 8 * (2 << 20)}


def med(counter):
    vals = {}
    for f in glob.glob(os.path.join(SRC, counter, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            k = next((k for k in KNOWN if k in row["Kernel_Name"]), None)
            if k:
                vals.setdefault(k, {}).setdefault(row["Dispatch_Id"], 0.0)
                vals[k][row["Dispatch_Id"]] += float(row["Counter_Value"]) * 1024
    return {k: statistics.median(v.values()) for k, v in vals.items()}


fetch, write = med("FETCH_SIZE"), med("WRITE_SIZE")
out = {}
for k, b in KNOWN.items():
    out[k] = {"known_bytes": b, "FETCH_SIZE_bytes": fetch.get(k), "WRITE_SIZE_bytes": write.get(k),
              "fetch_over_known": fetch[k] / b if k in fetch else None,
              "write_over_known": write[k] / b if k in write else None}
json.dump(out, sys.stdout, indent=1)
print()
