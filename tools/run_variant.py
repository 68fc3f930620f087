#!/usr/bin/env python3
"""Run ONE C2 launch configuration N times (for rocprofv3 --pmc passes; GPU box only).
Usage: python tools/run_variant.py <name> [reps]; names: pipe (kernel 2 default), stream (kernel 6),
probe (LDS-DMA read probe), probe_reg (register read probe)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "uc-tcp-ip_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED, c2_pseudo_headers  # noqa: E402
from sweep import set_tune  # noqa: E402

VARIANTS = {
    "pipe": dict(kernel=2, group=16, nt=1, tile=4),
    "stream": dict(kernel=6, k=4, nt=1, mult=4),
    "tile4": dict(kernel=4, group=16, nt=1, tile=4),
    "probe": dict(grid=8192, nt=1, probe=1),
    "probe_reg": dict(grid=8192, nt=1, probe=0),
}


def main():
    name = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    extra = dict(kv.split("=") for kv in sys.argv[3:])
    dev = torch.device("cuda", 0)
    n, L = 1 << 20, 1500
    seg = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(seg, n * L, SEED, 0)
    ph = torch.from_numpy(c2_pseudo_headers(0, n, L, 12)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    kw = dict(VARIANTS[name])
    kw.update({k: int(v) for k, v in extra.items()})
    set_tune(**kw)
    for _ in range(reps):
        if name.startswith("probe"):
            netcsum.read_stream(seg, n * L // 16 * 16, sink)
        else:
            netcsum.batch_strided(seg, L, L, ph, 12, 12, n, out, 0)
    torch.cuda.synchronize()
    print(name, kw, netcsum.last_launch())


if __name__ == "__main__":
    main()
