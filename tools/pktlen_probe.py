#!/usr/bin/env python3
"""Packed IPv4/TCP Rx batches (RxValidateIPv4, stride == total length) and uniform offset/length
segment batches (ChkSumBatchVarLen, packed) at datagram / segment lengths other than 1500 B, ≈ 1.5 GB
each, at the default launch and at other run lengths (NETCSUM_TUNE_TILE for Rx; for varlen batches
NETCSUM_TUNE_VARLEN_RUN_BYTES): do they fall into the run-byte cliffs of the dense segment stream
(runs whose bytes are a multiple of 16 KiB, or past 48 KiB; profiles/r6zq_seglen.jsonl)? GPU box only;
one JSON line per (kind, length, setting).
env: PLP_LENS (1024,2048,4096,8192,9000,1500), PLP_RX_RUNS (-1), PLP_VL_BYTES (-1), PLP_VL_TILES (-1:
none; fixed runs of that many segments), PLP_KINDS (rx,vl)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "tools", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED  # noqa: E402
from sweep import timeit  # noqa: E402


def main():
    lens = [int(x) for x in os.environ.get("PLP_LENS", "1024,2048,4096,8192,9000,1500").split(",")]
    rx_runs = [int(x) for x in os.environ.get("PLP_RX_RUNS", "-1").split(",")]
    vl_bytes = [int(x) for x in os.environ.get("PLP_VL_BYTES", "-1").split(",")]
    vl_tiles = [int(x) for x in os.environ.get("PLP_VL_TILES", "-1").split(",")]   # fixed runs (TUNE_TILE)
    kinds = os.environ.get("PLP_KINDS", "rx,vl").split(",")
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    for L in lens:
        n = int(1.5e9 // L)
        seg = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(seg, n * L, SEED, 0)
        if "rx" in kinds:
            v = seg[: n * L].view(n, L)
            v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
            flags = torch.zeros(n, dtype=torch.uint8, device=dev)
            netcsum.tx_finalize_ipv4(seg, n, flags, stride=L, pkt_len=L, stream=st)
            torch.cuda.synchronize()
            for r in rx_runs:
                netcsum.tune(netcsum.TUNE_TILE, r)
                fn = lambda: netcsum.rx_validate_ipv4(seg, n, flags, stride=L, pkt_len=L, stream=st)  # noqa: E731
                med, mn = timeit(fn, st, reps=50, warm_s=0.3)
                ok = bool((flags == 1).all().item()) if flags.dtype == torch.uint8 else None
                algo = n * (L + 1)
                print(json.dumps({"kind": "rx", "len": L, "n": n, "run": r, "kernel": netcsum.last_launch(),
                                  "ms": round(med, 4), "frac_of_8TBps": round(algo / med / 8e9, 4),
                                  "all_flags_1": ok}), flush=True)
            netcsum.tune(netcsum.TUNE_TILE, -1)
            del flags
        if "vl" in kinds:
            off = torch.from_numpy((np.arange(n, dtype=np.uint64) * np.uint64(L)).view(np.int64)).to(dev)
            ln = torch.from_numpy(np.full(n, L, np.uint16).view(np.int16)).to(dev)
            ph = torch.zeros(n * 12, dtype=torch.uint8, device=dev)
            out = torch.empty(n, dtype=torch.int16, device=dev)
            for b, t in [(b, -1) for b in vl_bytes] + [(-1, t) for t in vl_tiles if t > 0]:
                netcsum.tune(netcsum.TUNE_VARLEN_RUN_BYTES, b)
                netcsum.tune(netcsum.TUNE_TILE, t)
                fn = lambda: netcsum.batch_varlen(seg, off, ln, ph, 12, 12, n, out, 0, stream=st)  # noqa: E731
                med, mn = timeit(fn, st, reps=50, warm_s=0.3)
                algo = n * (L + 14)
                print(json.dumps({"kind": "varlen", "len": L, "n": n, "run_bytes": b, "tile": t, "kernel": netcsum.last_launch(),
                                  "ms": round(med, 4), "frac_of_8TBps": round(algo / med / 8e9, 4)}), flush=True)
            netcsum.tune(netcsum.TUNE_VARLEN_RUN_BYTES, -1)
            netcsum.tune(netcsum.TUNE_TILE, -1)
            del off, ln, ph, out
        del seg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
