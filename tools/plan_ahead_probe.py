#!/usr/bin/env python3
"""The first batch on a layout, with and without the ahead-sampler:
for each layout (1 M frames / segments), the wall time of one call + stream synchronisation on a
FRESH plan id (NetUtil_MI355X_PlanBind) with NETCSUM_TUNE_PLAN_AHEAD 0 (the batch runs unplanned and
samples for the next one) and 1 (a one-block sampler launch first, the call waits for its plan word),
and on a planned id (steady state), interleaved, median of R calls each. GPU box only; JSON lines.
  rings:  ring_mixed (40 / 576 / 1500 B in 1520-B slots), ring_tmpl (1500 B in 1520-B slots)
  pools:  pool1520mix, pool1520 (tools/varlen_pool_probe.py layouts)"""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "tools", ""):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
import ring_layouts  # noqa: E402


def main():
    n = int(os.environ.get("PLAN_N", 1 << 20))
    reps = int(os.environ.get("PLAN_REPS", 15))
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    cases = {}
    r = ring_layouts.mixed_ring(torch, netcsum, dev, n)
    f = torch.zeros(n, dtype=torch.uint8, device=dev)
    cases["ring_mixed"] = lambda r=r: netcsum.rx_validate_ipv4(r["base"], n, f, stride=1520, pkt_len=r["present"], stream=st)
    t = ring_layouts.uniform_ring(torch, netcsum, dev, n, 1520, 14)
    cases["ring_tmpl"] = lambda t=t: netcsum.rx_validate_ipv4(t["base"], n, f, stride=1520, pkt_len=t["present"], stream=st)
    rng = np.random.default_rng(5)
    offs = torch.from_numpy((np.arange(n, dtype=np.int64) * 1520 + 34)).to(dev)
    pbase = torch.empty(n * 1520 + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(pbase, n * 1520, 0x5EED0001, 0)
    ph = torch.from_numpy(rng.integers(0, 256, size=n * 12, dtype=np.uint8)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    for name, ln in (("pool1520mix", np.array([20, 556, 1480])[rng.choice(3, size=n, p=[7 / 12, 4 / 12, 1 / 12])]),
                     ("pool1520", np.full(n, 1480))):
        ld = torch.from_numpy(ln.astype(np.uint16).view(np.int16)).to(dev)
        cases[name] = lambda ld=ld: netcsum.batch_varlen(pbase, offs, ld, ph, 12, 12, n, out, 0, stream=st)
    torch.cuda.synchronize()
    pid = 1000
    res = {k: {"unplanned": [], "ahead": [], "planned": [], "desc": {}} for k in cases}
    # each case's planned id (the pool cases share their descriptor arrays' addresses: under one id
    # each would run in the other's plan)
    home = {name: 1 + i for i, name in enumerate(cases)}
    for name, fn in cases.items():                     # warm: each case's kernels and its planned id
        netcsum.plan_bind(home[name])
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
    for _ in range(reps):
        for name, fn in cases.items():
            for mode in ("unplanned", "ahead", "planned"):
                if mode == "planned":
                    netcsum.plan_bind(home[name])
                else:
                    pid += 1
                    netcsum.plan_bind(pid)
                netcsum.tune(netcsum.TUNE_PLAN_AHEAD, 1 if mode == "ahead" else 0)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                res[name][mode].append((time.perf_counter() - t0) * 1e3)
                res[name]["desc"][mode] = netcsum.last_launch()
    netcsum.tune(netcsum.TUNE_PLAN_AHEAD, -1)
    netcsum.plan_bind(0)
    for name, d in res.items():
        line = {"layout": name, "n": n}
        for mode in ("unplanned", "ahead", "planned"):
            line[f"{mode}_ms"] = round(statistics.median(d[mode]), 4)
            line[f"{mode}_kernel"] = d["desc"][mode]
        line["ahead_saves_ms"] = round(line["unplanned_ms"] - line["ahead_ms"], 4)
        line["ahead_over_planned_ms"] = round(line["ahead_ms"] - line["planned_ms"], 4)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
