#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace + FETCH_SIZE / WRITE_SIZE PMC collection of bench.py into
profiles/<tag>_pmc.json (read by bench.py for roofline.traffic).

HBM bytes per launch = FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024. FETCH_SIZE (KB) counts half of
the bytes of a 16-B/lane coalesced read stream on gfx950 (MI355X_MICROARCH.md §HBM; calibrated in
round 1: the read probe's FETCH_SIZE was exactly half of the bytes it read), hence the x2.
WRITE_SIZE reads exact for 16-B stores; our u16 stores are uncalibrated, listed separately."""
import csv
import json
import statistics
import sys
from collections import defaultdict


def kernel_rows(path, prefix):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].startswith(prefix) or prefix in r["Kernel_Name"]:
            d[r["Kernel_Name"]].append(r)
    return d


def main(tag, trace_dir, fetch_dir, write_dir, n_seg, bench_json=None, out_dir="profiles", seg_len=1500, plen=12):
    out = {"tag": tag, "n_seg": n_seg, "seg_len": seg_len, "pseudo_len": plen,
           "algorithmic_bytes_per_launch": n_seg * (seg_len + plen + 2)}
    if bench_json:                    # the launched kernel form + the hash of its sources (bench.py checks both)
        import os
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        kd = json.loads(open(bench_json).read().strip().splitlines()[-1])["roofline"]["kernel"]
        out["kernel_desc"] = kd
        out["kernel_src_sha"] = bench.kernel_src_sha(kd.split("::")[-1].split("<")[0])
    tr = kernel_rows(f"{trace_dir}/trace_kernel_trace.csv", "netcsum::")
    kern = {}
    for name, rows in tr.items():
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
        kern[name] = {"launches": len(rows), "avg_us": round(statistics.mean(durs), 2),
                      "median_us": round(statistics.median(durs), 2), "min_us": round(min(durs), 2),
                      "vgpr": rows[0]["VGPR_Count"], "lds": rows[0]["LDS_Block_Size"],
                      "grid": rows[0]["Grid_Size_X"], "wg": rows[0]["Workgroup_Size_X"]}
    out["kernel_trace"] = kern
    fetch = kernel_rows(f"{fetch_dir}/fetch_counter_collection.csv", "netcsum::")
    write = kernel_rows(f"{write_dir}/write_counter_collection.csv", "netcsum::")
    pmc = {}
    for name in set(fetch) | set(write):
        f = [float(r["Counter_Value"]) for r in fetch.get(name, []) if r["Counter_Name"] == "FETCH_SIZE"]
        w = [float(r["Counter_Value"]) for r in write.get(name, []) if r["Counter_Name"] == "WRITE_SIZE"]
        pmc[name] = {"FETCH_SIZE_KB": statistics.median(f) if f else None,
                     "WRITE_SIZE_KB": statistics.median(w) if w else None}
    out["pmc"] = pmc
    main_k = [k for k in pmc if "seg_" in k]
    if main_k:
        k = main_k[0]
        fb = pmc[k]["FETCH_SIZE_KB"] * 1024 * 2
        wb = pmc[k]["WRITE_SIZE_KB"] * 1024
        out["dominant_kernel"] = k
        out["hbm_read_bytes_per_launch"] = fb
        out["hbm_write_bytes_per_launch"] = wb
        out["hbm_bytes_per_launch"] = fb + wb
        out["traffic_over_algorithmic"] = round((fb + wb) / out["algorithmic_bytes_per_launch"], 4)
        tk = [v for n, v in kern.items() if "seg_" in n]
        if tk:
            out["rocprof_avg_us"] = tk[0]["avg_us"]
            out["achieved_GBps_from_rocprof_avg"] = round(out["algorithmic_bytes_per_launch"] / (tk[0]["avg_us"] * 1e3), 1)
    json.dump(out, open(f"{out_dir}/{tag}_pmc.json", "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]),
         sys.argv[6] if len(sys.argv) > 6 else None, sys.argv[7] if len(sys.argv) > 7 else "profiles")
