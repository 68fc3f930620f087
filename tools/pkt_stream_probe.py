#!/usr/bin/env python3
"""Rx / Tx packet-batch timing on 1 M x 1500-B IPv4/TCP datagrams (strided, in place):
the lane-group kernel (TUNE_KERNEL 2, tile 2) against the run-stream kernel over packets per wave
(TUNE_TILE), load policy (TUNE_NT_LOADS), pieces in flight (TUNE_CHUNKS 4 / 8) and the write-back
of the Tx field lines (TUNE_TX_FLUSH, env PS_FLUSH). Tx restores
nothing between launches: its written fields are the same every time. Prints JSON lines."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "tests", "tools", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED  # noqa: E402
from bench_configs import events_ms  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n, L = 1 << 20, 1500
    pk = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(pk, n * L, SEED, 0)
    v = pk[: n * L].view(n, L)
    v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
    flags8 = torch.zeros(8 * n, dtype=torch.uint8, device=dev)     # 8 B per packet: write-probe builds
    flags = flags8[:n]
    tx_flags = flags if os.environ.get("PS_TX_FLAGS") else None   # write-probe build 5 stores 8 B here
    ver = os.environ.get("PS_VER", "4")                          # 4, 6 or mix (alternating, bench_configs)
    rx_fn, tx_fn = netcsum.rx_validate_ipv4, netcsum.tx_finalize_ipv4
    if ver in ("6", "mix"):
        v[:, 0:8] = torch.tensor([0x60, 0, 0, 0, (L - 40) >> 8, (L - 40) & 0xFF, 6, 64], dtype=torch.uint8, device=dev)
        rx_fn, tx_fn = netcsum.rx_validate_ipv6, netcsum.tx_finalize_ipv6
        if os.environ.get("PS_CHAIN"):   # every datagram: a 200-B Destination Options header before TCP
            v[:, 6] = 60                  # (past every batch kernel's window: the walk pass's worst case)
            v[:, 40:42] = torch.tensor([6, 24], dtype=torch.uint8, device=dev)
        if ver == "mix":
            v[0::2, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8,
                                         device=dev)
            v[0::2, 12:20] = 0x0A
            rx_fn, tx_fn = netcsum.rx_validate_ip, netcsum.tx_finalize_ip
    tx_fn(pk, n, flags, stride=L, pkt_len=L, stream=st)
    torch.cuda.synchronize()
    variants = [] if os.environ.get("PS_NO_K2") else [dict(kernel=2, tile=2, nt=-1, chunks=0, passes=0)]
    for spw in [int(x) for x in os.environ.get("PS_SPW", "8,16,32").split(",")]:
        for nt in [int(x) for x in os.environ.get("PS_NT", "1,0").split(",")]:
            for d in [int(x) for x in os.environ.get("PS_D", "4,8").split(",")]:
                for passes in [int(x) for x in os.environ.get("PS_PASSES", "1,2").split(",")]:
                    for fl in [int(x) for x in os.environ.get("PS_FLUSH", "-1").split(",")]:
                        for w in [int(x) for x in os.environ.get("PS_WAVES", "-1").split(",")]:
                            variants.append(dict(kernel=0, tile=spw, nt=nt, chunks=d, passes=passes, flush=fl,
                                                 waves=w))
    for var in variants:
        netcsum.tune(netcsum.TUNE_TX_PASSES, var["passes"])
        netcsum.tune(netcsum.TUNE_TX_FLUSH, var.get("flush", -1))
        netcsum.tune(netcsum.TUNE_STREAM_WAVES, var.get("waves", -1))
        netcsum.tune(netcsum.TUNE_KERNEL, var["kernel"])
        netcsum.tune(netcsum.TUNE_TILE, var["tile"])
        netcsum.tune(netcsum.TUNE_NT_LOADS, var["nt"])
        netcsum.tune(netcsum.TUNE_CHUNKS, var["chunks"])
        res = {}
        for name, fn in (("rx", lambda: rx_fn(pk, n, flags, stride=L, pkt_len=L, stream=st)),
                         ("tx", lambda: tx_fn(pk, n, tx_flags, stride=L, pkt_len=L, stream=st))):
            ms = events_ms(fn, st, reps=60, warm_s=0.3)
            res[name] = {"ms": round(ms, 4), "GBps": round(n * (L + 1) / ms / 1e6, 1), "kernel": netcsum.last_launch()}
        ok = bool(((flags & 0x07) == 0x07).all()) if not os.environ.get("NETCSUM_LIB") else None
        print(json.dumps({"variant": var, "ver": ver, **res, "all_valid_after_tx": ok}), flush=True)


if __name__ == "__main__":
    main()
