#!/usr/bin/env python3
"""CRC-32 batch probe (net_util.c:485-636): the long-segment kernel forms side by side in one process
(NETCSUM_TUNE_CRC_KERNEL 1 = block combine, 2 = interleaved chunks, 3 = one lane per segment;
NETCSUM_TUNE_CRC_LANES, NETCSUM_TUNE_CRC_NT), interleaved
passes, every timed batch spot-checked against the oracle. One JSON line per (workload, variant).
    python tools/crc_probe.py [passes]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "tools", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
import oracle  # noqa: E402
from bench_configs import events_ms  # noqa: E402

SEED = 0x5EED0C3C
VARIANTS = ([{"kernel": 0, "nt": 0, "lanes": 0, "wide": 1}, {"kernel": 1, "nt": 0, "lanes": 0, "wide": 0},
             {"kernel": 3, "nt": 0, "lanes": 0, "wide": 0}]
            + [{"kernel": 2, "nt": 0, "lanes": g, "wide": w} for w in (1, 2) for g in (2, 4, 8, 16)])


def main():
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None      # e.g. "6,20": those lengths only
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    work = []
    # strided frames: (n, length, stride)
    for n, L, S in ((1 << 20, 1500, 1500), (1 << 20, 1514, 1518), (1 << 18, 9000, 9000), (1 << 22, 300, 300),
                    (1 << 22, 600, 600), (1 << 23, 64, 64), (1 << 23, 128, 128), (1 << 22, 256, 256),
                    (1 << 24, 6, 6), (1 << 24, 20, 20)):
        if only and str(L) not in only:
            continue
        buf = torch.empty(n * S + 64, dtype=torch.uint8, device=dev)
        netcsum.fill(buf, n * S, SEED, 0)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        work.append((f"strided {n} x {L} B (stride {S})", n * (L + 4),
                     (lambda b=buf, S=S, L=L, n=n, o=out: netcsum.crc32_strided(b, S, L, n, o, 1, stream=st)),
                     buf, out, dict(stride=S, length=L), n))
    # varlen: 1 M packed 40..3000-B segments at odd offsets
    rng = np.random.default_rng(5)
    nv = 1 << 20
    lens = rng.integers(40, 3000, size=nv).astype(np.uint32)
    off = np.zeros(nv, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    off += 1
    tot = int(off[-1] + lens[-1]) + 64
    vb = torch.empty(tot, dtype=torch.uint8, device=dev)
    netcsum.fill(vb, tot, SEED, 0)
    od = torch.from_numpy(off.view(np.int64)).to(dev)
    ld = torch.from_numpy(lens.view(np.int32)).to(dev)
    vo = torch.empty(nv, dtype=torch.int32, device=dev)
    work.append((f"varlen {nv} x 40..3000 B packed", int(lens.sum()) + nv * (12 + 4),
                 lambda: netcsum.crc32_varlen(vb, od, ld, nv, vo, 1, stream=st), vb, vo, dict(off=off, lens=lens), nv))
    res = {}
    for p in range(passes):
        for name, nbytes, fn, buf, out, lay, n in work:
            for v in VARIANTS:
                netcsum.tune(netcsum.TUNE_CRC_KERNEL, v["kernel"])
                netcsum.tune(netcsum.TUNE_CRC_NT, v["nt"])
                netcsum.tune(netcsum.TUNE_CRC_LANES, v["lanes"])
                netcsum.tune(netcsum.TUNE_CRC_WIDE, v["wide"])
                ms = events_ms(fn, st)
                key = (name, json.dumps(v))
                if p == 0:
                    idx = np.sort(np.random.default_rng(p).choice(n, 256, replace=False))
                    got = out.cpu().numpy().view(np.uint32)[idx]
                    if "stride" in lay:
                        S, L = lay["stride"], lay["length"]
                        rows = buf[: n * S].view(n, S)[torch.from_numpy(idx).to(dev)].cpu().numpy().reshape(-1)
                        want = oracle.crc32_batch(rows.copy(), len(idx), True, stride=S, length=L)
                    else:
                        host = buf.cpu().numpy()
                        want = oracle.crc32_batch(host, len(idx), True, off=lay["off"][idx], lens=lay["lens"][idx])
                    res[key] = {"same": bool(np.array_equal(got, want)), "ms": []}
                res[key]["ms"].append(ms)
                print(json.dumps({"work": name, "variant": v, "kernel": netcsum.last_launch(), "pass": p,
                                  "ms": round(ms, 4), "GB_per_s": round(nbytes / ms / 1e6, 1),
                                  "same": res[key]["same"]}), flush=True)
    netcsum.tune(netcsum.TUNE_CRC_KERNEL, 0)
    netcsum.tune(netcsum.TUNE_CRC_NT, 0)
    netcsum.tune(netcsum.TUNE_CRC_LANES, 0)
    netcsum.tune(netcsum.TUNE_CRC_WIDE, 1)


if __name__ == "__main__":
    main()
