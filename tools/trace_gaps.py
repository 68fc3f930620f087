#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (kernel_trace.csv): per kernel name the count and median
duration, and per consecutive (kernel -> next kernel) pair the median idle gap between them.
usage: python tools/trace_gaps.py <dir containing *kernel_trace.csv> [name filter]"""
import csv
import re
import glob
import statistics
import sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if flt in r["Kernel_Name"]]
dur, gap = defaultdict(list), defaultdict(list)
def short(s):
    s = re.sub(r"\(anonymous namespace\)::", "", s)
    s = re.sub(r"\([^()]*\)$", "", s.strip())          # the argument list
    return s.split("::")[-1][:60]
for a, b in zip(rows, rows[1:]):
    gap[(short(a["Kernel_Name"]), short(b["Kernel_Name"]))].append(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]))
for r in rows:
    dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in dur.items():
    print(f"kernel {k:60s} n={len(v):5d} median {statistics.median(v) / 1e3:8.2f} us")
for k, v in gap.items():
    if len(v) >= 20:
        print(f"gap {k[0]:40s} -> {k[1]:40s} n={len(v):5d} median {statistics.median(v) / 1e3:8.2f} us")
