#!/usr/bin/env python3
"""Strided batches of 256..1500-B segments with 12-B pseudo-headers (DataCalc): the default launch
policy against the run-stream segment kernel (TUNE_KERNEL 6) at several run lengths (TUNE_TILE) and
residencies, interleaved passes, results checked equal. GPU box only. JSON lines.
    SP_LENS=300,576 SP_TILES=16,32,54 SP_WAVES=-1,0 python tools/strided_probe.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED, c2_pseudo_headers  # noqa: E402
from bench_configs import events_ms  # noqa: E402


def env_list(k, default):
    return [int(x) for x in os.environ.get(k, default).split(",")]


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    for L in env_list("SP_LENS", "256,300,576,1000,1500"):
        n = (1_500_000_000 // L) & ~1023
        seg = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(seg, n * L, SEED, 0)
        ph = torch.from_numpy(c2_pseudo_headers(0, n, L, 12)).to(dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        algo = n * (L + 14)
        variants = [("default", 0, -1, -1)] + [(f"k6 tile {t} waves {w}", 6, t, w)
                                               for t in env_list("SP_TILES", "16,32,64") for w in env_list("SP_WAVES", "-1,0")]
        ref = None
        for p in range(int(os.environ.get("SP_PASSES", "2"))):
            for name, k, t, w in variants:
                netcsum.tune(netcsum.TUNE_KERNEL, k)
                netcsum.tune(netcsum.TUNE_TILE, t)
                netcsum.tune(netcsum.TUNE_STREAM_WAVES, w)
                fn = lambda: netcsum.batch_strided(seg, L, L, ph, 12, 12, n, out, 0, stream=st)  # noqa: E731
                ms = events_ms(fn, st, reps=20, warm_s=0.1)
                r = out.clone()
                same = True if ref is None else bool(torch.equal(r, ref))
                ref = r if ref is None else ref
                print(json.dumps({"len": L, "n": n, "pass": p, "variant": name, "kernel": netcsum.last_launch(),
                                  "ms": round(ms, 4), "GBps_algo": round(algo / ms / 1e6, 1), "same": same}), flush=True)
        netcsum.tune(netcsum.TUNE_KERNEL, 0)
        netcsum.tune(netcsum.TUNE_TILE, -1)
        netcsum.tune(netcsum.TUNE_STREAM_WAVES, -1)
        del seg, ph, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
