#!/usr/bin/env python3
"""C2 sweep: segmented-stream kernel (6) vs the pipelined lane-group kernel (2) and the read probes,
interleaved in one process (GPU box only). Prints one JSON line per variant."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "uc-tcp-ip_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED, c2_pseudo_headers  # noqa: E402
from sweep import set_tune, timeit  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
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
    variants = [("read", dict(grid=8192, nt=1, probe=1)), ("read", dict(grid=8192, nt=1, probe=0)),
                ("c2", dict(kernel=2, group=16, nt=1, tile=4))]
    spec = os.environ.get("SWEEP_STREAM", "4,6,8:1:1,2")
    ks, nts, mults = ([int(x) for x in part.split(",")] for part in spec.split(":"))
    for k in ks:
        for nt in nts:
            for mult in mults:
                variants.append(("c2", dict(kernel=6, k=k, nt=nt, mult=mult)))
    res = {}
    ref = None
    for r in range(rounds):
        for kind, kw in variants:
            set_tune(**kw)
            if kind == "read":
                fn = lambda: netcsum.read_stream(seg, n16, sink, stream=st)  # noqa: E731
                byts = n16
            else:
                fn = lambda: netcsum.batch_strided(seg, L, L, ph, 12, 12, n, out, 0, stream=st)  # noqa: E731
                byts = algo
            med, mn = timeit(fn, st, reps=30, warm_s=0.2)
            key = json.dumps([kind, kw], sort_keys=True)
            if kind == "c2":
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.clone()
                res.setdefault(key + "#same", []).append(bool(torch.equal(out, ref)))
                res.setdefault(key + "#launch", [netcsum.last_launch()])
            res.setdefault(key, []).append((med, mn, byts))
    set_tune()
    for key, v in res.items():
        if "#" in key:
            continue
        med = statistics.median(x[0] for x in v)
        mn = min(x[1] for x in v)
        byts = v[0][2]
        print(json.dumps({"variant": json.loads(key), "ms_med": round(med, 4), "ms_min": round(mn, 4),
                          "GBps_med": round(byts / med / 1e6, 1), "GBps_best": round(byts / mn / 1e6, 1),
                          "same_as_ref": all(res.get(key + "#same", [True])),
                          "launch": res.get(key + "#launch", [None])[0]}), flush=True)


if __name__ == "__main__":
    main()
