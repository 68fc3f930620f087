#!/usr/bin/env python3
"""C4 (1 M packed UDP datagrams of 40-9000 B, 12-B pseudo-headers, DataCalc) sweep of the varlen
run-stream kernel: segments per wave run (TUNE_TILE), pieces in flight (TUNE_CHUNKS) and resident
waves per SIMD (TUNE_STREAM_WAVES), interleaved passes, every variant checked equal to the first.
GPU box only. JSON lines.  C4_SPW=4,8,... C4_D=4,6 C4_WAVES=-1,4,6 C4_PASSES=2 python tools/c4_sweep.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED  # noqa: E402
from bench_configs import events_ms  # noqa: E402


def env_list(k, default):
    return [int(x) for x in os.environ.get(k, default).split(",")]


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 1 << 20
    lens = np.random.default_rng(7).integers(40, int(os.environ.get("C4_MAXLEN", "9000")) + 1, size=n).astype(np.uint16)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    total = int(off[-1]) + int(lens[-1])
    base = torch.empty(total + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(base, total, SEED, 0)
    off_d = torch.from_numpy(off.view(np.int64)).to(dev)
    len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
    ph = torch.from_numpy(np.random.default_rng(1).integers(0, 256, size=12 * n, dtype=np.uint8)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    algo = total + 14 * n
    ref = None
    if os.environ.get("C4_RUNB"):       # adaptive runs: target bytes per run (TILE left to the policy)
        variants = [(-1, 4, -1, b) for b in env_list("C4_RUNB", "0,8192,12288,16384,24576,32768")]
    else:
        variants = [(spw, d, w, 0) for spw in env_list("C4_SPW", "4,6,8,12,16") for d in env_list("C4_D", "4,6")
                    for w in env_list("C4_WAVES", "-1,4,6")]
    for p in range(int(os.environ.get("C4_PASSES", "2"))):
        for spw, d, w, rb in variants:
            netcsum.tune(netcsum.TUNE_VARLEN_RUN_BYTES, rb)
            netcsum.tune(netcsum.TUNE_TILE, spw)
            netcsum.tune(netcsum.TUNE_CHUNKS, d)
            netcsum.tune(netcsum.TUNE_STREAM_WAVES, w)
            fn = lambda: netcsum.batch_varlen(base, off_d, len_d, ph, 12, 12, n, out, 0, stream=st)  # noqa: E731
            ms = events_ms(fn, st, reps=20, warm_s=0.1)
            r = out.clone()
            same = True if ref is None else bool(torch.equal(r, ref))
            ref = r if ref is None else ref
            print(json.dumps({"pass": p, "variant": dict(spw=spw, d=d, waves=w, run_bytes=rb), "kernel": netcsum.last_launch(),
                              "ms": round(ms, 4), "GBps_algo": round(algo / ms / 1e6, 1), "same": same}), flush=True)
    netcsum.tune(netcsum.TUNE_TILE, -1)
    netcsum.tune(netcsum.TUNE_CHUNKS, 0)
    netcsum.tune(netcsum.TUNE_STREAM_WAVES, -1)
    netcsum.tune(netcsum.TUNE_VARLEN_RUN_BYTES, -1)


if __name__ == "__main__":
    main()
