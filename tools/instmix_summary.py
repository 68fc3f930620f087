#!/usr/bin/env python3
"""Per-kernel medians of the SQ counters of tools/gpu_instmix.sh runs. usage: instmix_summary.py DIR..."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "netcsum" in r["Kernel_Name"] and "fill_kernel" not in r["Kernel_Name"]:
                vals[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        print(d.split("/")[-1], k, {c: round(statistics.median(v)) for c, v in sorted(cs.items())})
