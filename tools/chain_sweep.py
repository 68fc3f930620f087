#!/usr/bin/env python3
"""Chain-batch launch sweep: the 16 Ki x 45-fragment reassembly batch of
tools/bench_configs.py, wave-per-chain kernel at several grid sizes vs the lane-group kernel,
every variant checked against the first. One JSON line per variant."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "tools", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED  # noqa: E402
from bench_configs import events_ms  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    nc, per, B = 1 << 14, 45, 2048
    plen = np.full(per, 1480, np.uint16)
    plen[-1] = 65515 - 1480 * (per - 1) - 8
    lens = np.tile(plen, nc)
    offs = (np.arange(nc * per, dtype=np.uint64) * B + 42).astype(np.uint64)
    first = (np.arange(nc + 1, dtype=np.uint64) * per).astype(np.uint32)
    base = torch.empty(nc * per * B + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(base, nc * per * B, SEED, 0)
    ph = np.zeros((nc, 12), np.uint8)
    ph[:, 9] = 17
    ph = torch.from_numpy(ph.reshape(-1)).to(dev)
    off_d = torch.from_numpy(offs.view(np.int64)).to(dev)
    len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
    first_d = torch.from_numpy(first.view(np.int32)).to(dev)
    oc = torch.empty(nc, dtype=torch.int16, device=dev)
    payload = int(lens.astype(np.int64).sum())
    ref = None
    for group, grid in [(0, 0), (0, 1024), (0, 2048), (0, 8192), (0, 16384), (32, 0), (32, 4096), (32, 8192)]:
        netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
        netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
        fn = lambda: netcsum.batch_chains(base, off_d, len_d, first_d, ph, 12, 12, nc, oc, 0, stream=st,  # noqa: E731
                                          n_pieces=nc * per)
        fn()
        torch.cuda.synchronize()
        if ref is None:
            ref = oc.clone()
        ms = events_ms(fn, st, reps=40)
        print(json.dumps({"variant": {"group": group, "grid": grid}, "ms_med": round(ms, 4),
                          "GiBps_checksummed": round((payload + 12 * nc) / ms / 1e6 / 1.073741824, 1),
                          "same": bool(torch.equal(oc, ref))}), flush=True)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, 0)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, 0)
    # Reference point: the same pieces as independent segments (no chaining, no pseudo-header) through
    # the segment-batch kernels — the practical read rate of this scattered 1480-of-2048-B layout.
    out = torch.empty(nc * per, dtype=torch.int16, device=dev)
    for kernel in (0, 2, 6):
        netcsum.tune(netcsum.TUNE_KERNEL, kernel)
        fn = lambda: netcsum.batch_varlen(base, off_d, len_d, None, 0, 0, nc * per, out, 0, stream=st)  # noqa: E731
        ms = events_ms(fn, st, reps=40)
        print(json.dumps({"variant": {"segments_kernel": kernel, "launch": netcsum.last_launch()},
                          "ms_med": round(ms, 4),
                          "GiBps_checksummed": round(payload / ms / 1e6 / 1.073741824, 1)}), flush=True)
    netcsum.tune(netcsum.TUNE_KERNEL, 0)


if __name__ == "__main__":
    main()
