#!/usr/bin/env python3
"""Tx finalize write-back sweep: 1 M x 1500-B IPv4/TCP datagrams, strided, in place.

For each variant (write-back form x nt x tile) the batch is restored from a pristine copy, finalized
once and compared byte-for-byte with the two-byte-store result (itself checked on a sample against
the packet oracle), then timed. Fused Rx over the same bytes is the no-store reference point.
Prints one JSON line per variant."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "tests", "tools", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
import oracle_packets as op  # noqa: E402
from bench import SEED  # noqa: E402
from bench_configs import events_ms  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n, L = 1 << 20, int(os.environ.get("TX_SWEEP_LEN", "1500"))
    pk = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(pk, n * L, SEED, 0)
    v = pk[: n * L].view(n, L)
    v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
    v[:, 36:38] = 0
    pristine = pk.clone()
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)

    netcsum.tx_finalize_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st)
    torch.cuda.synchronize()
    want = pk.clone()
    sel = np.arange(0, n, n // 128)
    src = pristine.cpu().numpy()
    dst = want.cpu().numpy()
    oracle_ok = all(bytes(dst[i * L:(i + 1) * L]) == op.tx_finalize(bytes(src[i * L:(i + 1) * L]), True)[0]
                    for i in sel.tolist())
    ms_rx = events_ms(lambda: netcsum.rx_validate_ipv4(want, n, flags, stride=L, pkt_len=L, stream=st), st, reps=40)
    print(json.dumps({"variant": "rx_fused", "ms_med": round(ms_rx, 4),
                      "GBps_med": round(n * L / ms_rx / 1e6, 1), "oracle_sample_ok": oracle_ok}), flush=True)
    groups = [int(g) for g in os.environ.get("TX_SWEEP_GROUPS", "0").split(",")]
    wbs = [0]
    for g in groups:
        netcsum.tune(netcsum.TUNE_GROUP_LANES, g)
        if g:
            ms_g = events_ms(lambda: netcsum.rx_validate_ipv4(want, n, flags, stride=L, pkt_len=L, stream=st), st,
                             reps=40)
            print(json.dumps({"variant": {"rx_group": g}, "ms_med": round(ms_g, 4),
                              "GBps_med": round(n * L / ms_g / 1e6, 1)}), flush=True)
        grids = [int(x) for x in os.environ.get("TX_SWEEP_GRIDS", "0").split(",")]
        tiles = [int(x) for x in os.environ.get("TX_SWEEP_TILES", "1,2,4").split(",")]
        nts = [int(x) for x in os.environ.get("TX_SWEEP_NT", "1,0").split(",")]
        for wb, nt, tile, grid in [(w, t, j, q) for w in wbs for t in nts for j in tiles for q in grids]:
                netcsum.tune(netcsum.TUNE_NT_LOADS, nt)
                netcsum.tune(netcsum.TUNE_TILE, tile)
                netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
                pk.copy_(pristine)
                netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st)
                torch.cuda.synchronize()
                same = bool(torch.equal(pk, want))
                ms = events_ms(lambda: netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st), st,
                               reps=40)
                print(json.dumps({"variant": {"group": g, "wb": wb, "nt": nt, "tile": tile, "grid": grid},
                                  "ms_med": round(ms, 4),
                                  "GBps_med": round(n * (L + 4) / ms / 1e6, 1), "same_as_first": same}),
                      flush=True)
    for k, val in ((netcsum.TUNE_NT_LOADS, -1), (netcsum.TUNE_TILE, -1),
                   (netcsum.TUNE_GROUP_LANES, 0), (netcsum.TUNE_GRID_BLOCKS, 0)):
        netcsum.tune(k, val)


if __name__ == "__main__":
    main()
