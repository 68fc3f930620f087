#!/usr/bin/env python3
"""Why does the run-stream packet kernel (Rx, 1 M x 1500-B IPv4/TCP) read faster than the C2
segment kernel over the same number of bytes? Interleaves, in one process on one
1 M x 1500-B buffer: C2 as bench.py runs it (12-B pseudo-headers from memory), C2 without
pseudo-headers, C2 Verify (1-B results) (C2P_FORMS), each at several segments per wave (C2P_SPW) and
residency caps (C2P_WAVES, NETCSUM_TUNE_STREAM_WAVES), pieces in flight (C2P_D) and with / without
the row touch (C2P_TOUCH),
C4 (C2P_FORMS c4), the Rx packet kernel on the same bytes made
IPv4/TCP, and the read probes. GPU box only; prints JSON lines."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "tests", "tools", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED, c2_pseudo_headers  # noqa: E402
from sweep import set_tune, timeit  # noqa: E402


def main():
    rounds = int(os.environ.get("C2P_ROUNDS", "3"))
    spws = [int(x) for x in os.environ.get("C2P_SPW", "8,16,32").split(",")]
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n, L = int(os.environ.get("C2P_N", 1 << 20)), 1500
    seg = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(seg, n * L, SEED, 0)
    v = seg[: n * L].view(n, L)          # IPv4/TCP headers: the C2 kernels do not care, Rx needs them
    v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
    ph = torch.from_numpy(c2_pseudo_headers(0, n, L, 12)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    netcsum.tx_finalize_ipv4(seg, n, flags, stride=L, pkt_len=L, stream=st)
    torch.cuda.synchronize()
    n16 = n * L // 16 * 16

    def c2(pseudo, op):
        if pseudo:
            return lambda: netcsum.batch_strided(seg, L, L, ph, 12, 12, n, out, op, stream=st)
        return lambda: netcsum.batch_strided(seg, L, L, None, 0, 0, n, out, op, stream=st)

    c4 = None
    forms = os.environ.get("C2P_FORMS", "calc_pseudo,rx").split(",")
    if "c4" in forms:                        # C4 as tools/bench_configs.py builds it (seed 7, 40..9000 B)
        import numpy as np
        rng = np.random.default_rng(7)
        nv = 1 << 20
        lens = rng.integers(40, 9001, size=nv).astype(np.uint16)
        off = np.zeros(nv, np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        tot = int(off[-1]) + int(lens[-1])
        base4 = torch.empty(tot + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(base4, tot, SEED, 0)
        off_d = torch.from_numpy(off.view(np.int64)).to(dev)
        len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
        ph4 = torch.zeros(nv * 12, dtype=torch.uint8, device=dev)
        o4 = torch.empty(nv, dtype=torch.int16, device=dev)
        c4 = (lambda: netcsum.batch_varlen(base4, off_d, len_d, ph4, 12, 12, nv, o4, 0, stream=st), tot + nv * 14)
    variants = [("read_lds", dict(grid=8192, nt=1, probe=1), (-1, -1, -1), lambda: netcsum.read_stream(seg, n16, sink, stream=st), n16),
                ("read_reg", dict(grid=8192, nt=1, probe=0), (-1, -1, -1), lambda: netcsum.read_stream(seg, n16, sink, stream=st), n16)]
    touches = [int(x) for x in os.environ.get("C2P_TOUCH", "-1").split(",")]
    depths = [int(x) for x in os.environ.get("C2P_D", "0").split(",")]
    xcds = [int(x) for x in os.environ.get("C2P_XCD", "-1").split(",")]
    for w, spw, tch, dd, xc in [(w, spw, t, dd, xc) for w in [int(x) for x in os.environ.get("C2P_WAVES", "-1").split(",")]
                                for spw in spws for t in touches for dd in depths for xc in xcds]:
            sfx = f"_spw{spw}_waves{w}_touch{tch}" + (f"_D{dd}" if dd else "") + (f"_xcd{xc}" if xc >= 0 else "")
            if c4 is not None:
                variants.append(("c4" + sfx, dict(kernel=6, tile=spw, k=dd), (w, tch, xc), c4[0], c4[1]))
            if "calc_pseudo" in forms:
                variants.append(("c2_calc_pseudo" + sfx, dict(kernel=6, tile=spw, k=dd), (w, tch, xc), c2(True, 0), n * (L + 12 + 2)))
            if "calc_nopseudo" in forms:
                variants.append(("c2_calc_nopseudo" + sfx, dict(kernel=6, tile=spw), (w, tch, xc), c2(False, 0), n * (L + 2)))
            if "verify_pseudo" in forms:
                variants.append(("c2_verify_pseudo" + sfx, dict(kernel=6, tile=spw), (w, tch, xc), c2(True, 1), n * (L + 12 + 1)))
            if "rx" in forms:
                variants.append(("rx_pkt" + sfx, dict(tile=spw), (w, tch, xc),
                                 lambda: netcsum.rx_validate_ipv4(seg, n, flags, stride=L, pkt_len=L, stream=st), n * (L + 1)))
    res = {}
    for _ in range(rounds):
        for name, kw, (w, tch, xc), fn, byts in variants:
            set_tune(**kw)
            netcsum.tune(netcsum.TUNE_STREAM_WAVES, w)
            netcsum.tune(netcsum.TUNE_STREAM_TOUCH, tch)
            netcsum.tune(netcsum.TUNE_STREAM_XCD, xc)
            med, mn = timeit(fn, st, reps=40, warm_s=0.3)
            res.setdefault(name, []).append((med, mn, byts, netcsum.last_launch()))
    set_tune()
    netcsum.tune(netcsum.TUNE_STREAM_WAVES, -1)
    netcsum.tune(netcsum.TUNE_STREAM_TOUCH, -1)
    netcsum.tune(netcsum.TUNE_STREAM_XCD, -1)
    for name, r in res.items():
        med = statistics.median(x[0] for x in r)
        print(json.dumps({"variant": name, "kernel": r[0][3], "ms_med": round(med, 4),
                          "ms_min": round(min(x[1] for x in r), 4), "GBps_med": round(r[0][2] / med / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
