#!/usr/bin/env python3
"""Launch-option sweep of the packet run-stream kernel on 1 M x 1500-B IPv4/TCP datagrams (fused Rx
and two-pass Tx): resident waves per SIMD (TUNE_STREAM_WAVES), the row touch (TUNE_STREAM_TOUCH),
the XCD-aware block order (TUNE_STREAM_XCD) and packets per run (TUNE_TILE), two interleaved passes;
every variant's Rx flags must all be valid. One JSON line per (pass, variant)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "", "tools"):
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
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st)
    variants = []
    for waves in (-1, 5, 6):
        for touch in (-1, 1):
            for xcd in (-1, 1):
                for tile in (-1, 16):
                    variants.append((waves, touch, xcd, tile))
    for rep in range(2):
        for waves, touch, xcd, tile in variants:
            netcsum.tune(netcsum.TUNE_STREAM_WAVES, waves)
            netcsum.tune(netcsum.TUNE_STREAM_TOUCH, touch)
            netcsum.tune(netcsum.TUNE_STREAM_XCD, xcd)
            netcsum.tune(netcsum.TUNE_TILE, tile)
            rx = events_ms(lambda: netcsum.rx_validate_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st), st)
            ok = bool(((flags & 0x07) == 0x07).all().item())
            tx = events_ms(lambda: netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st), st)
            print(json.dumps({"pass": rep, "waves": waves, "touch": touch, "xcd": xcd, "tile": tile,
                              "rx_ms": round(rx, 4), "tx_ms": round(tx, 4), "rx_all_valid": ok}), flush=True)
    for k in (netcsum.TUNE_STREAM_WAVES, netcsum.TUNE_STREAM_TOUCH, netcsum.TUNE_STREAM_XCD, netcsum.TUNE_TILE):
        netcsum.tune(k, -1)


if __name__ == "__main__":
    main()
