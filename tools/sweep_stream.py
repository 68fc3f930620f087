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
    if os.environ.get("SWEEP_C3"):
        return sweep_c3(rounds, dev, st)
    if os.environ.get("SWEEP_C4"):
        return sweep_c4(rounds, dev, st)
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


def sweep_c3(rounds, dev, st):
    """C3: 16 M x 20 B IPv4 headers, HdrCalc: kernel 5 (register loads) vs kernel 7 (LDS tiles)."""
    nh = 1 << 24
    hdr = torch.empty(nh * 20 + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(hdr, nh * 20, SEED, 0)
    o3 = torch.empty(nh, dtype=torch.int16, device=dev)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    nb = nh * 20 // 16 * 16
    variants = [("read", dict(grid=8192, nt=1, probe=1)), ("c3", dict(kernel=5))]
    c3spec = os.environ.get("SWEEP_C3_SPEC", "2,3,4:1,2,4:-1")     # stages : grid mults : headers per lane
    parts = c3spec.split(":") + ["-1"] * (3 - len(c3spec.split(":")))
    c3k, c3m, c3h = ([int(x) for x in part.split(",")] for part in parts)
    for h in c3h:
        for k in c3k:
            for mult in c3m:
                variants.append(("c3", dict(kernel=7, k=k, mult=mult, tile=h)))
    res, ref = {}, None
    for r in range(rounds):
        for kind, kw in variants:
            set_tune(**kw)
            if kind == "read":
                fn = lambda: netcsum.read_stream(hdr, nb, sink, stream=st)  # noqa: E731
                byts = nb
            else:
                fn = lambda: netcsum.batch_strided(hdr, 20, 20, None, 0, 0, nh, o3, 2, stream=st)  # noqa: E731
                byts = nh * 22
            med, mn = timeit(fn, st, reps=30, warm_s=0.2)
            key = json.dumps([kind, kw], sort_keys=True)
            if kind == "c3":
                torch.cuda.synchronize()
                if ref is None:
                    ref = o3.clone()
                res.setdefault(key + "#same", []).append(bool(torch.equal(o3, ref)))
                res.setdefault(key + "#launch", [netcsum.last_launch()])
            res.setdefault(key, []).append((med, mn, byts))
    set_tune()
    for key, v in res.items():
        if "#" in key:
            continue
        med = statistics.median(x[0] for x in v)
        print(json.dumps({"variant": json.loads(key), "ms_med": round(med, 4), "GBps_med": round(v[0][2] / med / 1e6, 1),
                          "Ghdr_per_s": round(nh / med / 1e6, 2), "same_as_ref": all(res.get(key + "#same", [True])),
                          "launch": res.get(key + "#launch", [None])[0]}), flush=True)


def sweep_c4(rounds, dev, st):
    """C4: 1 M packed UDP datagrams 40..9000 B (seed 7) + 12 B pseudo: kernel 2 vs kernel 6."""
    import numpy as np
    rng = np.random.default_rng(7)
    nv = 1 << 20
    lens = rng.integers(40, 9001, size=nv).astype(np.uint16)
    off = np.zeros(nv, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    if os.environ.get("SWEEP_C4_RING"):                  # NIC-ring layout: one 9216-B buffer per datagram
        off = np.arange(nv, dtype=np.uint64) * 9216 + 42
    tot = int(off[-1]) + int(lens[-1])
    base = torch.empty(tot + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(base, tot, SEED, 0)
    off_d = torch.from_numpy(off.view(np.int64)).to(dev)
    len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
    ph4 = torch.randint(0, 256, (nv * 12,), dtype=torch.uint8, device=dev)
    o4 = torch.empty(nv, dtype=torch.int16, device=dev)
    variants = [("c4", dict(kernel=2, group=32, k=8, nt=1, tile=4))]
    spec = os.environ.get("SWEEP_C4_SPEC", "4,8:8,16,32,64")
    ks, runs = ([int(x) for x in part.split(",")] for part in spec.split(":"))
    for k in ks:
        for run in runs:
            variants.append(("c4", dict(kernel=6, k=k, tile=run, nt=1)))
    res, ref = {}, None
    byts = int(lens.astype(np.uint64).sum()) + nv * (12 + 2)
    for r in range(rounds):
        for kind, kw in variants:
            set_tune(**kw)
            fn = lambda: netcsum.batch_varlen(base, off_d, len_d, ph4, 12, 12, nv, o4, 0, stream=st)  # noqa: E731
            med, mn = timeit(fn, st, reps=20, warm_s=0.2)
            key = json.dumps([kind, kw], sort_keys=True)
            torch.cuda.synchronize()
            if ref is None:
                ref = o4.clone()
            res.setdefault(key + "#same", []).append(bool(torch.equal(o4, ref)))
            res.setdefault(key + "#launch", [netcsum.last_launch()])
            res.setdefault(key, []).append((med, mn))
    set_tune()
    for key, v in res.items():
        if "#" in key:
            continue
        med = statistics.median(x[0] for x in v)
        print(json.dumps({"variant": json.loads(key), "ms_med": round(med, 4), "GBps_med": round(byts / med / 1e6, 1),
                          "GiBps_checksummed": round((byts - 2 * nv) / med / 1e6 / 1.073741824, 1),
                          "same_as_ref": all(res.get(key + "#same", [True])),
                          "launch": res.get(key + "#launch", [None])[0]}), flush=True)


if __name__ == "__main__":
    main()
