#!/usr/bin/env python3
"""C3 (16 M x 20-B IPv4 headers, HdrCalc) sweep of seg_hdr_kernel<P,S,H>: headers per lane H (TILE),
tiles in flight S (CHUNKS), grid (GRID_BLOCKS; 0 = tiles / 16 = 4 tiles per wave), and of the
run-stream header kernel 8 over headers per run (C3_SPW), residency cap (C3_WAVES) and row touch
(C3_TOUCH), against the LDS-DMA read probe over the same 335 MB. Results checked equal across
variants. JSON lines."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED  # noqa: E402
from bench_configs import events_ms  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n, L = 1 << 24, 20
    hdr = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(hdr, n * L, SEED, 0)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    algo = n * (L + 2)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, 8192)
    ms = events_ms(lambda: netcsum.read_stream(hdr, n * L, sink, stream=st), st, reps=40, warm_s=0.3)
    print(json.dumps({"variant": "read_probe", "ms": round(ms, 4), "GBps": round(n * L / ms / 1e6, 1)}), flush=True)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, 0)
    ref = None
    spws = [int(x) for x in os.environ.get("C3_SPW", "384,512,768,1024").split(",")]
    waves_l = [int(x) for x in os.environ.get("C3_WAVES", "-1").split(",")]
    touch_l = [int(x) for x in os.environ.get("C3_TOUCH", "-1").split(",")]
    xcd_l = [int(x) for x in os.environ.get("C3_XCD", "-1").split(",")]
    d_l = [int(x) for x in os.environ.get("C3_D", "4,8").split(",")]
    burst_l = [int(x) for x in os.environ.get("C3_BURST", "-1").split(",")]
    passes = int(os.environ.get("C3_PASSES", "1"))
    for spw, d, nt, w, tch, xc, bu in [(spw, d, nt, w, t, xc, bu) for _ in range(passes) for spw in spws for d in d_l
                                       for nt in (1,) for w in waves_l for t in touch_l for xc in xcd_l for bu in burst_l]:
                netcsum.tune(netcsum.TUNE_HDR_BURST, bu)
                netcsum.tune(netcsum.TUNE_STREAM_XCD, xc)
                netcsum.tune(netcsum.TUNE_STREAM_WAVES, w)
                netcsum.tune(netcsum.TUNE_STREAM_TOUCH, tch)
                netcsum.tune(netcsum.TUNE_KERNEL, 8)
                netcsum.tune(netcsum.TUNE_TILE, spw)
                netcsum.tune(netcsum.TUNE_CHUNKS, d)
                netcsum.tune(netcsum.TUNE_NT_LOADS, nt)
                fn = lambda: netcsum.batch_strided(hdr, L, L, None, 0, 0, n, out, 2, stream=st)  # noqa: E731
                ms = events_ms(fn, st, reps=40, warm_s=0.2)
                r = out.clone()
                same = True if ref is None else bool(torch.equal(r, ref))
                ref = r if ref is None else ref
                print(json.dumps({"variant": dict(kernel=8, spw=spw, d=d, nt=nt, waves=w, touch=tch, xcd=xc, burst=bu),
                                  "kernel": netcsum.last_launch(),
                                  "ms": round(ms, 4), "GBps_algo": round(algo / ms / 1e6, 1), "same": same}), flush=True)
    netcsum.tune(netcsum.TUNE_NT_LOADS, -1)
    netcsum.tune(netcsum.TUNE_STREAM_WAVES, -1)
    netcsum.tune(netcsum.TUNE_STREAM_TOUCH, -1)
    netcsum.tune(netcsum.TUNE_STREAM_XCD, -1)
    netcsum.tune(netcsum.TUNE_HDR_BURST, -1)
    if os.environ.get("C3_NO_K7"):
        return
    for h in (2, 4):
        for s in (2, 3, 4):
            if h == 4 and s == 4:
                continue
            for div in (0, 8):
                tiles = n // (64 * h)
                grid = 0 if div == 0 else tiles // div
                netcsum.tune(netcsum.TUNE_KERNEL, 7)
                netcsum.tune(netcsum.TUNE_TILE, h)
                netcsum.tune(netcsum.TUNE_CHUNKS, s)
                netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
                fn = lambda: netcsum.batch_strided(hdr, L, L, None, 0, 0, n, out, 2, stream=st)  # noqa: E731
                ms = events_ms(fn, st, reps=40, warm_s=0.2)
                r = out.clone()
                same = True if ref is None else bool(torch.equal(r, ref))
                ref = r if ref is None else ref
                print(json.dumps({"variant": dict(h=h, s=s, tiles_per_wave=(div or 16) // 4 if div else 4, grid=grid),
                                  "kernel": netcsum.last_launch(), "ms": round(ms, 4),
                                  "GBps_algo": round(algo / ms / 1e6, 1), "same": same}), flush=True)
    for k in (netcsum.TUNE_KERNEL, netcsum.TUNE_CHUNKS, netcsum.TUNE_GRID_BLOCKS):
        netcsum.tune(k, 0)
    netcsum.tune(netcsum.TUNE_TILE, -1)


if __name__ == "__main__":
    main()
