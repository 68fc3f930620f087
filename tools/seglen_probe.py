#!/usr/bin/env python3
"""Dense strided segment batches (the C2 form: stride == len, 12-B IPv4 pseudo-headers, DataCalc) at
segment lengths other than C2's 1500 B — MSS-sized TCP segments (1448 / 1460), jumbo frames, powers of
two — ≈ 1.5 GB each, at the library's default launch (runs of 16 segments, row touch, 5 waves per
SIMD) and, with SLP_RUNS, at other run lengths (NETCSUM_TUNE_TILE): does any common length fall off
the rate C2 reaches? Run lengths near C2's default showed a 15 % cliff one segment away
(profiles/r6zo_c2_runs.log). GPU box only; one JSON line per (length, run).
env: SLP_LENS (default 1024,1280,1448,1460,1472,1480,1500,1514,2048,4096,8192,9000), SLP_RUNS (-1),
SLP_BYTES (1.5e9)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "tools", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED, c2_pseudo_headers  # noqa: E402
from sweep import timeit  # noqa: E402


def main():
    lens = [int(x) for x in os.environ.get("SLP_LENS", "1024,1280,1448,1460,1472,1480,1500,1514,2048,4096,8192,9000").split(",")]
    runs = [int(x) for x in os.environ.get("SLP_RUNS", "-1").split(",")]
    total = float(os.environ.get("SLP_BYTES", "1.5e9"))
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    for L in lens:
        n = int(total // L)
        seg = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(seg, n * L, SEED, 0)
        ph = torch.from_numpy(c2_pseudo_headers(0, n, L, 12)).to(dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        for r in runs:
            netcsum.tune(netcsum.TUNE_TILE, r)
            fn = lambda: netcsum.batch_strided(seg, L, L, ph, 12, 12, n, out, 0, stream=st)  # noqa: E731
            med, mn = timeit(fn, st, reps=50, warm_s=0.3)
            algo = n * (L + 12 + 2)
            print(json.dumps({"len": L, "n": n, "run": r, "kernel": netcsum.last_launch(), "ms": round(med, 4),
                              "ms_min": round(mn, 4), "GB_per_s_algorithmic": round(algo / med / 1e6, 1),
                              "frac_of_8TBps": round(algo / med / 8e9, 4)}), flush=True)
        netcsum.tune(netcsum.TUNE_TILE, -1)
        del seg, ph, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
