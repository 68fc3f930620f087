#!/usr/bin/env python3
"""Host-side enqueue cost of one batch launch through the Python binding (GPU box): time N async
launches without synchronising, then the drain. If enqueue/launch < kernel time the GPU never idles."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED, c2_pseudo_headers  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
n, L = 1 << 20, 1500
seg = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
netcsum.fill(seg, n * L, SEED, 0)
ph = torch.from_numpy(c2_pseudo_headers(0, n, L, 12)).to(dev)
out = torch.empty(n, dtype=torch.int16, device=dev)
res = {}
for steps in (100, 400):
    for rep in range(3):
        for _ in range(20):
            netcsum.batch_strided(seg, L, L, ph, 12, 12, n, out, 0, stream=st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            netcsum.batch_strided(seg, L, L, ph, 12, 12, n, out, 0, stream=st)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res.setdefault(str(steps), []).append({"enqueue_us_per_launch": round((t1 - t0) / steps * 1e6, 2),
                                               "wall_ms_per_step": round((t2 - t0) / steps * 1e3, 5)})
print(json.dumps(res))
