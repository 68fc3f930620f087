#!/usr/bin/env python3
"""Launch-geometry sweep for the checksum kernels and the read-stream probe (GPU box only).

Interleaves variants in ONE process (cdna_hip_programming.md §5.4 rule 24) and prints the
median/min HIP-event time per variant as JSON lines. Config: C2 (1 M x 1500 B + 12 B pseudo) by
default; --c3 adds 16 M x 20 B headers, --c4 adds 1 M packed 40-9000 B UDP datagrams.
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "uc-tcp-ip_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED, c2_pseudo_headers  # noqa: E402


def timeit(fn, stream, reps=20, warm=3, warm_s=0.1):
    t0 = time.perf_counter()                     # warm by time (clock ramp after idle gaps)
    k = 0
    while k < warm or time.perf_counter() - t0 < warm_s:
        fn()
        k += 1
        if k % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    ts = [a.elapsed_time(b) for a, b in ev]
    return statistics.median(ts), min(ts)


def set_tune(grid=0, group=0, nt=-1, block=0, kernel=0, k=0, probe=1, mult=0, tile=-1):
    netcsum.tune(netcsum.TUNE_GRID_MULT, mult)
    netcsum.tune(netcsum.TUNE_TILE, tile)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    netcsum.tune(netcsum.TUNE_NT_LOADS, nt)
    netcsum.tune(netcsum.TUNE_BLOCK_THREADS, block)
    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
    netcsum.tune(netcsum.TUNE_CHUNKS, k)
    netcsum.tune(netcsum.TUNE_PROBE, probe)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c3", action="store_true")
    ap.add_argument("--c4", action="store_true")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--no-c2", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n, L = 1 << 20, 1500
    seg = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(seg, n * L, SEED, 0)
    ph = torch.from_numpy(c2_pseudo_headers(0, n, L, 12)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    n16 = n * L // 16 * 16
    algo = n * (L + 12 + 2)

    variants = []
    for probe in (0, 1):
        variants.append(("read", dict(grid=8192, nt=1, probe=probe)))
    for group in (8, 16, 32):
        for tile, grid in ((1, 0), (2, 0), (4, 0), (8, 0), (0, 8192), (0, 16384), (0, 32768)):
            variants.append(("c2", dict(kernel=2, group=group, nt=1, grid=grid, tile=tile)))
    for block in (128, 64):
        variants.append(("c2", dict(kernel=2, group=16, nt=1, block=block, tile=4)))
    variants.append(("c2", dict(kernel=2, group=16, nt=0, tile=4)))
    variants.append(("c2", dict(kernel=3, group=16, nt=1, tile=4)))
    variants.append(("c2", dict(kernel=4, group=16, nt=1, tile=4)))
    res = {}
    if args.no_c2:
        variants = []
    for r in range(args.rounds):
        for kind, kw in variants:
            set_tune(**kw)
            if kind == "read":
                fn = lambda: netcsum.read_stream(seg, n16, sink, stream=st)  # noqa: E731
                byts = n16
            else:
                fn = lambda: netcsum.batch_strided(seg, L, L, ph, 12, 12, n, out, 0, stream=st)  # noqa: E731
                byts = algo
            med, mn = timeit(fn, st)
            key = json.dumps([kind, kw], sort_keys=True)
            res.setdefault(key, []).append((med, mn, byts))
    set_tune()
    for key, v in res.items():
        med = statistics.median(x[0] for x in v)
        mn = min(x[1] for x in v)
        byts = v[0][2]
        print(json.dumps({"variant": json.loads(key), "ms_med": round(med, 4), "ms_min": round(mn, 4),
                          "GBps_med": round(byts / med / 1e6, 1), "GBps_best": round(byts / mn / 1e6, 1)}), flush=True)

    if args.c3:
        nh = 1 << 24
        hdr = torch.empty(nh * 20 + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(hdr, nh * 20, SEED, 0)
        o3 = torch.empty(nh, dtype=torch.int16, device=dev)
        for probe in (0, 1):
            set_tune(grid=8192, nt=1, probe=probe)
            nb = nh * 20 // 16 * 16
            med, mn = timeit(lambda: netcsum.read_stream(hdr, nb, sink, stream=st), st)
            print(json.dumps({"variant": ["c3-read", dict(probe=probe)], "ms_med": round(med, 4),
                              "GBps_med": round(nb / med / 1e6, 1)}), flush=True)
        for kernel, group, k, nt in ((2, 1, 2, 0), (5, 0, 0, 0)):
            for grid, tile in ((8192, 0), (16384, 0), (0, 1), (0, 2), (0, 4), (0, 8), (0, 16)):
                set_tune(grid=grid, group=group, kernel=kernel, k=k, nt=nt, tile=tile)
                med, mn = timeit(lambda: netcsum.batch_strided(hdr, 20, 20, None, 0, 0, nh, o3, 2, stream=st), st)
                b = nh * (20 + 2)
                print(json.dumps({"variant": ["c3", dict(kernel=kernel, group=group, k=k, nt=nt, grid=grid, tile=tile)], "ms_med": round(med, 4),
                                  "GBps_med": round(b / med / 1e6, 1), "Mhdr_per_s": round(nh / med / 1e3, 1)}),
                      flush=True)
        set_tune()
    if args.c4:
        rng = np.random.default_rng(7)
        nv = 1 << 20
        lens = rng.integers(40, 9001, size=nv).astype(np.uint16)
        off = np.zeros(nv, np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        tot = int(off[-1]) + int(lens[-1])
        base = torch.empty(tot + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(base, tot, SEED, 0)
        off_d = torch.from_numpy(off.view(np.int64)).to(dev)
        len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
        ph4 = torch.zeros(nv * 12, dtype=torch.uint8, device=dev)
        o4 = torch.empty(nv, dtype=torch.int16, device=dev)
        for kernel, group, k in ((2, 32, 8), (2, 32, 6), (2, 64, 4), (2, 16, 8)):
            for grid, tile in ((16384, 0), (0, 1), (0, 2), (0, 4)):
                set_tune(grid=grid, group=group, kernel=kernel, k=k, nt=1, tile=tile)
                med, mn = timeit(lambda: netcsum.batch_varlen(base, off_d, len_d, ph4, 12, 12, nv, o4, 0, stream=st), st)
                b = tot + nv * (12 + 2)
                print(json.dumps({"variant": ["c4", dict(kernel=kernel, group=group, k=k, grid=grid, tile=tile)], "ms_med": round(med, 4),
                                  "GBps_med": round(b / med / 1e6, 1), "GiBps_checksummed": round((tot + 12 * nv) / med / 1e6 / 1.073741824, 1)}),
                      flush=True)
        set_tune()


if __name__ == "__main__":
    main()
