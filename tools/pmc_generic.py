#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc output directories of any counters: per directory, per kernel (name up
to its template arguments' end), the median per launch of every counter collected, and the launch
count. Usage: python tools/pmc_generic.py OUT.json LABEL=DIR [LABEL=DIR ...]
The kernel-source hash of the segment stream (bench.kernel_src_sha) is recorded beside the numbers."""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def summarise(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in vals.items():
        out[k] = {c: statistics.median(v) for c, v in cs.items()}
        out[k]["launches"] = max(len(v) for v in cs.values())
    return out


def main():
    import bench
    res = {"kernel_src_sha": {"seg_stream_kernel": bench.kernel_src_sha("seg_stream_kernel")}, "passes": {}}
    for arg in sys.argv[2:]:
        label, d = arg.split("=", 1)
        res["passes"][label] = summarise(d)
    json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
