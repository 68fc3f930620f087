#!/usr/bin/env python3
"""Packet run-stream kernel (fused Rx validate / Tx finalize of strided IPv4/TCP datagrams): run
length (TUNE_TILE = datagrams per wave run) against datagram length, interleaved passes, Rx verdicts
checked all-valid after a Tx finalize. GPU box only. JSON lines.
    PR_LENS=128,576,1500 PR_TILES=8,16,32,64 python tools/pkt_run_probe.py"""
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


def env_list(k, default):
    return [int(x) for x in os.environ.get(k, default).split(",")]


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    for L in env_list("PR_LENS", "128,256,576,1000,1500"):
        n = (1_500_000_000 // L) & ~1023
        pk = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(pk, n * L, SEED, 0)
        v = pk[: n * L].view(n, L)
        v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
        v[:, 32] = 0x50                                   # TCP data offset 5 (20-B header)
        flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st)
        for p in range(int(os.environ.get("PR_PASSES", "2"))):
            for t in env_list("PR_TILES", "-1,8,16,32,64"):      # -1: the library's default
                netcsum.tune(netcsum.TUNE_TILE, t)
                for op in ("rx", "tx"):
                    if op == "rx":
                        fn = lambda: netcsum.rx_validate_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st)  # noqa: E731
                    else:
                        fn = lambda: netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st)  # noqa: E731
                    ms = events_ms(fn, st, reps=20, warm_s=0.1)
                    ok = None
                    if op == "rx":
                        ok = bool((flags == 0x07).all())         # IP_OK | L4_OK | L4_CHECKED
                    print(json.dumps({"len": L, "n": n, "pass": p, "op": op, "tile": t, "kernel": netcsum.last_launch(),
                                      "ms": round(ms, 4), "GBps": round(n * L / ms / 1e6, 1), "all_valid": ok}), flush=True)
        netcsum.tune(netcsum.TUNE_TILE, -1)
        del pk, v, flags
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
