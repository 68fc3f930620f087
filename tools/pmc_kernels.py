#!/usr/bin/env python3
"""Summarise tools/gpu_pmc.sh output for one config: per netcsum kernel the rocprofv3 kernel-trace
average duration and the FETCH_SIZE / WRITE_SIZE PMC per launch (median), HBM bytes per launch
= FETCH_SIZE x 1024 x 2 (gfx950 correction for 16-B/lane streaming reads, MI355X_MICROARCH.md §HBM)
+ WRITE_SIZE x 1024, and the ratio to the algorithmic bytes tools/run_config.py printed."""
import csv
import glob
import json
import re
import statistics
import sys
from collections import defaultdict


def rows(pattern):
    f = glob.glob(pattern, recursive=True)
    if not f:
        return []
    return list(csv.DictReader(open(f[0])))


# the source file that defines each kernel (+ the shared headers): a summary is evidence for the
# exact sources whose hash it records
KERNEL_FILES = {"seg_stream": "netcsum_stream.hip", "seg_live": "netcsum_stream.hip", "seg_pipe": "netcsum_kernels.hip", "pkt_vl_deferred": "netcsum_pktstream.hip", "read_run": "netcsum_stream.hip", "varlen_runlen": "netcsum_stream.hip",
                "seg_hdrstream": "netcsum_hdrstream.hip", "seg_hdr_": "netcsum_hdr.hip", "pkt_stream": "netcsum_pktstream.hip",
                "pkt_scatter": "netcsum_pktstream.hip", "pkt_batch": "netcsum_packets.hip", "pkt_v6_walk": "netcsum_v6walk.hip",
                "chain_": "netcsum_chains.hip", "crc_": "netcsum_crc.hip", "seg_small": "netcsum_small.hip"}
COMMON = ["netcsum_device.h", "netcsum_kernels.h", "netcsum_stream.h"]


def src_sha(kernel_name):
    import hashlib
    import os
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "uc-tcp-ip_amd", "csrc")
    f = next((v for k, v in KERNEL_FILES.items() if k in kernel_name), None)
    if f is None:
        return None
    h = hashlib.sha256()
    for name in [f] + COMMON:
        h.update(open(os.path.join(csrc, name), "rb").read())
    return h.hexdigest()[:16]


def main(tag, cfg, out):
    log = open(f"{out}/{tag}_{cfg}_run.log").read()
    m = re.search(r"algo_bytes=(\d+)", log)
    algo = int(m.group(1)) if m else None
    m = re.search(r"reps=(\d+)", log)
    reps = int(m.group(1)) if m else None
    trace = defaultdict(list)
    for r in sorted(rows(f"{out}/{tag}_{cfg}_trace/**/trace_kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"])):
        if "netcsum" in r["Kernel_Name"]:
            trace[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if reps:                                            # the timed launches only (after the warm-up)
        trace = defaultdict(list, {k: (v[-reps:] if len(v) > reps else v) for k, v in trace.items()})
    pmc = defaultdict(dict)
    for kind, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        vals = defaultdict(list)
        for r in rows(f"{out}/{tag}_{cfg}_{kind}/**/{kind}_counter_collection.csv"):
            if "netcsum" in r["Kernel_Name"] and r["Counter_Name"] == ctr:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        for k, v in vals.items():
            pmc[k][ctr + "_KB"] = statistics.median(v)
    extra = defaultdict(lambda: defaultdict(list))     # optional third pass (EXTRA_PMC)
    for r in rows(f"{out}/{tag}_{cfg}_extra/**/extra_counter_collection.csv"):
        if "netcsum" in r["Kernel_Name"]:
            extra[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in extra.items():
        for c, v in cs.items():
            pmc[k][c] = statistics.median(v)
    res = {"tag": tag, "config": cfg, "launch": next((ln for ln in log.splitlines() if ln.startswith(cfg + " ")), None),
           "algorithmic_bytes_per_launch": algo, "kernels": {}}
    for k in sorted(set(trace) | set(pmc)):
        d = {"launches": len(trace.get(k, [])),
             "avg_us": round(statistics.mean(trace[k]), 2) if trace.get(k) else None,
             "min_us": round(min(trace[k]), 2) if trace.get(k) else None, **pmc.get(k, {})}
        if "FETCH_SIZE_KB" in d and "WRITE_SIZE_KB" in d:
            d["hbm_read_bytes"] = d["FETCH_SIZE_KB"] * 1024 * 2
            d["hbm_write_bytes"] = d["WRITE_SIZE_KB"] * 1024
            if algo:
                d["traffic_over_algorithmic"] = round((d["hbm_read_bytes"] + d["hbm_write_bytes"]) / algo, 4)
        if algo and d["avg_us"]:
            d["algorithmic_GBps_at_avg"] = round(algo / (d["avg_us"] * 1e3), 1)
        d["kernel_src_sha"] = src_sha(k)
        res["kernels"][k] = d
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
