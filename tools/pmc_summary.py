"""Summarise rocprofv3 PMC passes (gpurun_out/prof_<tag>/pmc*/...) per kernel dispatch."""
import collections
import csv
import glob
import os
import sys

tag = sys.argv[1]
root = tag if os.path.isdir(tag) else f"gpurun_out/prof_{tag}"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in sorted(glob.glob(f"{root}/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "cbx::" not in k and "cbx_jit" not in k:
            continue
        key = (os.path.basename(os.path.dirname(f)), r["Dispatch_Id"])
        names[key] = k.split("(")[0]
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
for key in sorted(agg, key=lambda k: (k[0], int(k[1]))):
    print(key[0], key[1], names[key], {c: int(v) for c, v in sorted(agg[key].items())})
