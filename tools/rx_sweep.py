#!/usr/bin/env python3
"""Launch-geometry sweep of the fused IPv4 Rx validation / Tx finalize kernels on 1 M x 1500 B TCP
datagrams (valid checksums), next to the segment kernel on the same bytes. One JSON line per point."""
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
    netcsum.tx_finalize_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st)
    torch.cuda.synchronize()
    out = torch.empty(n, dtype=torch.int16, device=dev)
    gb = n * L / 1e9
    ms = events_ms(lambda: netcsum.batch_strided(pk, L, L, None, 0, 0, n, out, 0, stream=st), st)
    print(json.dumps({"kernel": netcsum.last_launch(), "what": "seg DataCalc 1500B", "ms": round(ms, 4),
                      "GBps": round(gb / ms * 1e3, 1)}), flush=True)
    for tx in (False, True):
        for g in (8, 16, 32, 64):
            for grid, tile in ((0, -1), (0, 1), (0, 2), (0, 8), (4096, 0), (16384, 0)):
                netcsum.tune(netcsum.TUNE_GROUP_LANES, g)
                netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
                netcsum.tune(netcsum.TUNE_TILE, tile)
                if tx:
                    fn = lambda: netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st)  # noqa: E731
                else:
                    fn = lambda: netcsum.rx_validate_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st)  # noqa: E731
                ms = events_ms(fn, st, reps=10)
                ok = bool(((flags & 0x07) == 0x07).all().item()) if not tx else None
                print(json.dumps({"what": "tx" if tx else "rx", "G": g, "grid": grid, "tile": tile,
                                  "ms": round(ms, 4), "GBps": round(gb / ms * 1e3, 1), "all_valid": ok}), flush=True)
    for k in (netcsum.TUNE_GROUP_LANES, netcsum.TUNE_GRID_BLOCKS):
        netcsum.tune(k, 0)
    netcsum.tune(netcsum.TUNE_TILE, -1)


if __name__ == "__main__":
    main()
