#!/usr/bin/env python3
"""Round 6, verdict r5 item 1: where does the C5 shard (16 M x 1500 B + 12 B, 25.4 GB) lose its
per-GPU rate against C2 (1 M, 1.6 GB) on some boxes? Interleaves, in one process, on the C5 shard
and on a C2 batch allocated beside it (GPU box only; JSON lines):
  kernel            the library's default launch (bench.py's step)
  nopseudo          the same segments without pseudo-headers (no second address stream)
  chunk1M           the 16 M segments as 16 back-to-back launches of 1 M (C2-sized footprints)
  run_probe         read_run_kernel: the kernel's access pattern, nothing computed (TUNE_PROBE 2)
  lds_probe         the LDS-DMA grid-stride read probe (TUNE_PROBE 1)
  touch0 / xcd0     the kernel without the row touch / in the plain block order
  gather0           the kernel with each wave storing its own results (round 5's partial-line stores)
  d6 / d8           6 / 8 pieces in flight per wave (NETCSUM_TUNE_CHUNKS)
  w4 / w6 / w8      4 / 6 / 8 resident waves per SIMD (NETCSUM_TUNE_STREAM_WAVES; default 5)
  s8 / s24 / s32    runs of 8 / 24 / 32 segments (NETCSUM_TUNE_TILE; default 16)
  run_probe_sleep   read_run_kernel with a ~128-clock pause after each piece (TUNE_PROBE 3)
  alloc2 / alloc2_run_probe   the kernel / its read probe on a SECOND 25-GB allocation of the same shard
  onealloc          the kernel with the pseudo-headers and the results inside the segments' allocation
  seg1_out2 / seg2_out1 / seg1_ph2_out2   the first allocations' buffers crossed with the second's
  run_probe_x1      the read probe in the kernel's XCD-slice block order (the probe's default: dispatch order)
  x4 / x16 / x64 / x128 / x256 / x1024 / x4096   the kernel with XCD chunks of C blocks in turn
                    (NETCSUM_TUNE_STREAM_XCD C); xcd1 the one-slice-per-XCD order; run_probe_x256 the probe
  alloc2_xcd0 / alloc2_x16  the second allocation in the plain / chunked block order
Median / min of C5P_REPS HIP-event-timed launches per variant, C5P_ROUNDS interleaved rounds."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "tools", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED, c2_pseudo_headers  # noqa: E402
from sweep import timeit  # noqa: E402


def main():
    rounds = int(os.environ.get("C5P_ROUNDS", "3"))
    reps = int(os.environ.get("C5P_REPS", "20"))
    only = os.environ.get("C5P_VARIANTS")
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    L, P = 1500, 12
    sizes = {"c5": 1 << 24, "c2": 1 << 20}
    bufs = {}
    for name, n in sizes.items():
        seg = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(seg, n * L, SEED, 0)
        ph = torch.from_numpy(c2_pseudo_headers(0, n, L, P)).to(dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        bufs[name] = (n, seg, ph, out)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    extra = []
    if not only or any(x.startswith("alloc2") or x == "onealloc" or x.startswith("seg") for x in only.split(",")):
        n = sizes["c5"]
        seg2 = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(seg2, n * L, SEED, 0)
        ph2 = bufs["c5"][2].clone()
        out2 = torch.empty(n, dtype=torch.int16, device=dev)
        big = torch.empty(n * L + 256 + n * P + 256 + 2 * n, dtype=torch.uint8, device=dev)   # one allocation
        segb = big[: n * L + 256]
        netcsum.fill(segb, n * L, SEED, 0)
        phb = big[n * L + 256: n * L + 256 + n * P]
        phb.copy_(bufs["c5"][2])
        o0 = n * L + 256 + n * P + 256
        outb = big[o0: o0 + 2 * n].view(torch.int16)
        n5 = n                                   # (bound now: the loop below rebinds n)
        extra = [("c5_alloc2", {}, lambda: netcsum.batch_strided(seg2, L, L, ph2, P, P, n5, out2, netcsum.OP_DATA_CALC, stream=st),
                  n5 * (L + P + 2)),
                 ("c5_alloc2_run_probe", {"probe": 2}, lambda: netcsum.read_stream(seg2, n5 * L // 16 * 16, sink, stream=st),
                  n5 * L // 16 * 16),
                 ("c5_alloc2_run_probe_x1", {"probe": 2, "xcd": 1},
                  lambda: netcsum.read_stream(seg2, n5 * L // 16 * 16, sink, stream=st), n5 * L // 16 * 16),
                 ("c5_onealloc", {}, lambda: netcsum.batch_strided(segb, L, L, phb, P, P, n5, outb, netcsum.OP_DATA_CALC, stream=st),
                  n5 * (L + P + 2)),
                 # which buffer of the first allocations carries the loss: crossed pairs
                 ("c5_seg1_out2", {}, lambda: netcsum.batch_strided(bufs["c5"][1], L, L, bufs["c5"][2], P, P, n5, out2,
                                                                    netcsum.OP_DATA_CALC, stream=st), n5 * (L + P + 2)),
                 ("c5_seg2_out1", {}, lambda: netcsum.batch_strided(seg2, L, L, ph2, P, P, n5, bufs["c5"][3],
                                                                    netcsum.OP_DATA_CALC, stream=st), n5 * (L + P + 2)),
                 ("c5_alloc2_xcd0", {"xcd": 0}, lambda: netcsum.batch_strided(seg2, L, L, ph2, P, P, n5, out2,
                                                                    netcsum.OP_DATA_CALC, stream=st), n5 * (L + P + 2)),
                 ("c5_alloc2_x16", {"xcd": 16}, lambda: netcsum.batch_strided(seg2, L, L, ph2, P, P, n5, out2,
                                                                  netcsum.OP_DATA_CALC, stream=st), n5 * (L + P + 2)),
                 ("c5_seg1_ph2_out2", {}, lambda: netcsum.batch_strided(bufs["c5"][1], L, L, ph2, P, P, n5, out2,
                                                                        netcsum.OP_DATA_CALC, stream=st), n5 * (L + P + 2))]
    torch.cuda.synchronize()

    def tune(probe=1, touch=-1, xcd=-1, gather=-1, d=0, waves=-1, tile=-1):
        netcsum.tune(netcsum.TUNE_TILE, tile)
        netcsum.tune(netcsum.TUNE_CHUNKS, d)
        netcsum.tune(netcsum.TUNE_STREAM_WAVES, waves)
        netcsum.tune(netcsum.TUNE_PROBE, probe)
        netcsum.tune(netcsum.TUNE_STREAM_TOUCH, touch)
        netcsum.tune(netcsum.TUNE_STREAM_XCD, xcd)
        netcsum.tune(netcsum.TUNE_STORE_GATHER, gather)

    variants = []
    for name, (n, seg, ph, out) in bufs.items():
        n16 = n * L // 16 * 16
        algo = n * (L + P + 2)

        def k(seg=seg, ph=ph, out=out, n=n):
            return lambda: netcsum.batch_strided(seg, L, L, ph, P, P, n, out, netcsum.OP_DATA_CALC, stream=st)

        def nop(seg=seg, out=out, n=n):
            return lambda: netcsum.batch_strided(seg, L, L, None, 0, 0, n, out, netcsum.OP_DATA_CALC, stream=st)

        def chunked(seg=seg, ph=ph, out=out, n=n):
            m = 1 << 20
            parts = [(seg[i * m * L:], ph[i * m * P:], out[i * m:]) for i in range(n // m)]

            def f():
                for s, p, o in parts:
                    netcsum.batch_strided(s, L, L, p, P, P, m, o, netcsum.OP_DATA_CALC, stream=st)
            return f

        def rd(seg=seg, n16=n16):
            return lambda: netcsum.read_stream(seg, n16, sink, stream=st)
        variants += [(f"{name}_kernel", {}, k(), algo), (f"{name}_nopseudo", {}, nop(), n * (L + 2)),
                     (f"{name}_run_probe", {"probe": 2}, rd(), n16), (f"{name}_lds_probe", {"probe": 1}, rd(), n16),
                     (f"{name}_touch0", {"touch": 0}, k(), algo), (f"{name}_xcd0", {"xcd": 0}, k(), algo),
                     (f"{name}_gather0", {"gather": 0}, k(), algo), (f"{name}_d6", {"d": 6}, k(), algo),
                     (f"{name}_d8", {"d": 8}, k(), algo), (f"{name}_w4", {"waves": 4}, k(), algo),
                     (f"{name}_w6", {"waves": 6}, k(), algo), (f"{name}_w8", {"waves": 8}, k(), algo),
                     (f"{name}_s8", {"tile": 8}, k(), algo),
                     (f"{name}_s24", {"tile": 24}, k(), algo), (f"{name}_s32", {"tile": 32}, k(), algo),
                     (f"{name}_run_probe_sleep", {"probe": 3}, rd(), n16),
                     (f"{name}_x4", {"xcd": 4}, k(), algo), (f"{name}_x16", {"xcd": 16}, k(), algo),
                     (f"{name}_x64", {"xcd": 64}, k(), algo), (f"{name}_x256", {"xcd": 256}, k(), algo),
                     (f"{name}_x128", {"xcd": 128}, k(), algo), (f"{name}_x1024", {"xcd": 1024}, k(), algo),
                     (f"{name}_x4096", {"xcd": 4096}, k(), algo), (f"{name}_xcd1", {"xcd": 1}, k(), algo),
                     (f"{name}_run_probe_x256", {"probe": 2, "xcd": 256}, rd(), n16),
                     (f"{name}_run_probe_x1", {"probe": 2, "xcd": 1}, rd(), n16)]
        if n > (1 << 20):
            variants.append((f"{name}_chunk1M", {}, chunked(), algo))
    variants += extra
    if only:
        keep = only.split(",")
        variants = [v for v in variants if any(v[0].endswith(x) for x in keep)]
    res = {}
    for _ in range(rounds):
        for name, kw, fn, byts in variants:
            tune(**kw)
            med, mn = timeit(fn, st, reps=reps, warm_s=0.3)
            res.setdefault(name, []).append((med, mn, byts, netcsum.last_launch()))
    tune()
    for name, r in res.items():
        med = statistics.median(x[0] for x in r)
        print(json.dumps({"variant": name, "kernel": r[0][3], "ms_med": round(med, 4),
                          "ms_min": round(min(x[1] for x in r), 4), "GBps_med": round(r[0][2] / med / 1e6, 1),
                          "frac_of_8TBps": round(r[0][2] / med / 1e6 / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
