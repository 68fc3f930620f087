#!/usr/bin/env python3
"""Does segment alignment (partial 128-B lines per wave-instruction) limit the kernels?
Times the C2 kernel at segment lengths 1500 / 1504 / 1536 / 1024 / 2048 (stride = length) and a
pure-read LDS-DMA probe, interleaved in one process."""
import json, os, statistics, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "uc-tcp-ip_amd")); sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa
import netcsum  # noqa
from sweep import timeit, set_tune  # noqa
from bench import SEED  # noqa

dev = torch.device("cuda", 0); st = torch.cuda.current_stream(dev)
TOT = 1 << 20
buf = torch.empty(TOT * 2048 + 4096, dtype=torch.uint8, device=dev)
netcsum.fill(buf, buf.numel() - 8, SEED, 0)
NMAX = (1500 * TOT) // 1024                      # most segments of any tested length
ph = torch.zeros(NMAX * 12 + 64, dtype=torch.uint8, device=dev)
out = torch.empty(NMAX, dtype=torch.int16, device=dev)
sink = torch.zeros(1, dtype=torch.int64, device=dev)
res = {}
for rnd in range(2):
    for L in (1500, 1504, 1536, 1024, 2048):
        n = (1500 * TOT) // L
        assert n <= NMAX and n * L <= buf.numel()
        for kernel, group, k, grid in ((2, 16, 6, 16384), (3, 16, 6, 0), (2, 16, 8, 16384), (2, 32, 4, 16384), (3, 32, 4, 0), (2, 64, 2, 16384)):
            if L == 2048 and group == 16 and k == 6:
                k = 8
            set_tune(kernel=kernel, group=group, k=k, nt=1, grid=grid)
            med, mn = timeit(lambda: netcsum.batch_strided(buf, L, L, ph, 12, 12, n, out, 0, stream=st), st)
            res.setdefault((L, kernel, group, k, grid), []).append((med, n * (L + 14)))
    set_tune(probe=1, nt=1, grid=8192)
    nb = 1500 * TOT // 16 * 16
    med, mn = timeit(lambda: netcsum.read_stream(buf, nb, sink, stream=st), st)
    res.setdefault(("probe_lds",), []).append((med, nb))
set_tune()
for k, v in res.items():
    med = statistics.median(x[0] for x in v)
    print(json.dumps({"variant": list(k), "ms": round(med, 4), "GBps": round(v[0][1] / med / 1e6, 1)}))
