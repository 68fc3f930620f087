#!/usr/bin/env python3
"""ChkSumBatchVarLen over TCP segments where the stack holds them: inside NET_BUF pool buffers, at
DataPtr + TransportHdrIx (net_util.c:1627-1628,1649; net_tcp.c:1920), one segment per buffer (GPU box
only).

Layouts (1 M segments, a 12-B IPv4 pseudo-header each, offsets in buffer order):
  pool1520     1480-B segments (1500-B datagrams) at +34 of 1520-B buffers (the template's large
               buffers, Cfg/Template/net_dev_cfg.c:146-148: Ethernet 14 + IPv4 20)
  pool1520mix  segments of 20 / 556 / 1480 B (40 / 576 / 1500-B datagrams at 7 : 4 : 1) there
  pool2k       1480-B segments at +84 of 2048-B buffers (IPv4 header at +64)
  pool2kmix    the mix there
  c4           BASELINE configs[3] for comparison: 40-9000 B packed back to back (not a pool layout)
each under the default launch and the variants named on stdout (TUNE_KERNEL 2: the lane-group pipe at
16 lanes x 6 chunks). Median HIP-event time of 20 launches after a warm-up, two interleaved passes;
the segment bytes (+ 12 B pseudo + 2 B out per segment) over the time, fraction of 8 TB/s. A 4096-
segment sample of the default's outputs is checked against the oracle.

  python tools/varlen_pool_probe.py [layout ...] > gpurun_out/TAG_varlen_pool_probe.jsonl
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
from ring_probe import events_ms  # noqa: E402

LAYOUTS = {"pool1520": (1520, 34, False), "pool1520mix": (1520, 34, True), "pool2k": (2048, 84, False),
           "pool2kmix": (2048, 84, True), "c4": (0, 0, False)}
VARIANTS = [("default", {}), ("pipe16", {netcsum.TUNE_KERNEL: 2, netcsum.TUNE_GROUP_LANES: 16, netcsum.TUNE_CHUNKS: 6}),
            ("runs8", {netcsum.TUNE_VARLEN_RUN_BYTES: 0}),
            ("pieces", {netcsum.TUNE_LIVE_COMPACT: 0})]   # round 6: the live pieces, not the compacted sectors
if os.environ.get("POOL_LIVE"):                       # live-sector stream: run length x pieces in flight
    for r, dd in ((8, 4), (8, 8), (16, 4), (16, 8), (24, 4), (24, 8), (32, 4), (32, 8), (40, 4), (40, 8)):
        VARIANTS.append((f"live.s{r}.d{dd}", {netcsum.TUNE_TILE: r, netcsum.TUNE_CHUNKS: dd}))
if os.environ.get("POOL_PIPES"):                      # lane-group pipe geometries (kernel 2)
    for g, k, t in ((16, 6, 2), (16, 6, 8), (16, 6, 16), (32, 4, 4), (8, 8, 4), (16, 8, 4)):
        VARIANTS.append((f"pipe{g}k{k}t{t}", {netcsum.TUNE_KERNEL: 2, netcsum.TUNE_GROUP_LANES: g,
                                              netcsum.TUNE_CHUNKS: k, netcsum.TUNE_TILE: t}))
RESET = {netcsum.TUNE_KERNEL: 0, netcsum.TUNE_GROUP_LANES: 0, netcsum.TUNE_CHUNKS: 0, netcsum.TUNE_VARLEN_RUN_BYTES: -1,
         netcsum.TUNE_TILE: -1, netcsum.TUNE_LIVE_COMPACT: -1}


def main():
    import oracle
    n = int(os.environ.get("POOL_N", 1 << 20))
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    want = sys.argv[1:] or list(LAYOUTS)
    extra = [v for v in os.environ.get("POOL_VARIANTS", "").split(",") if v]
    for name in want:
        slot, ix, mix = LAYOUTS[name]
        rng = np.random.default_rng(5)
        if slot == 0:                                  # C4: packed 40-9000 B
            lens = rng.integers(40, 9001, size=n).astype(np.uint16)
            offs = np.zeros(n, np.uint64)
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
            total = int(offs[-1]) + int(lens[-1])
        else:
            lens = (np.array([20, 556, 1480])[rng.choice(3, size=n, p=[7 / 12, 4 / 12, 1 / 12])] if mix
                    else np.full(n, 1480)).astype(np.uint16)
            offs = (np.arange(n, dtype=np.uint64) * np.uint64(slot) + np.uint64(ix)).astype(np.uint64)
            total = n * slot
        base = torch.empty(total + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(base, total // 8 * 8, 0x5EED0001, 0)
        ph = torch.from_numpy(rng.integers(0, 256, size=n * 12, dtype=np.uint8)).to(dev)
        off_d = torch.from_numpy(offs.view(np.int64)).to(dev)
        len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        seg_bytes = int(lens.astype(np.int64).sum())
        algo = seg_bytes + n * (12 + 2)
        res = {}
        for p in range(2):
            for tag, knobs in VARIANTS + [(v, {}) for v in extra]:
                for k, v in knobs.items():
                    netcsum.tune(k, v)
                ms = events_ms(lambda: netcsum.batch_varlen(base, off_d, len_d, ph, 12, 12, n, out, netcsum.OP_DATA_CALC,
                                                            stream=st), st)
                d = res.setdefault(tag, {"ms": [], "kernel": netcsum.last_launch()})
                d["kernel"] = netcsum.last_launch()                 # (the plan the timed calls ran)
                d["ms"].append(ms)
                if tag == "default" and p == 0:
                    torch.cuda.synchronize()
                    smp = np.sort(rng.choice(n, size=4096, replace=False))
                    got = out.cpu().numpy().view(np.uint16)[smp]
                    hb = base.cpu().numpy()
                    segs = np.concatenate([hb[int(offs[i]):int(offs[i]) + int(lens[i])] for i in smp])
                    so = np.zeros(len(smp), np.uint64)
                    so[1:] = np.cumsum(lens[smp][:-1].astype(np.uint64))
                    phs = ph.cpu().numpy().reshape(n, 12)[smp].reshape(-1)
                    d["parity_sample_ok"] = bool(np.array_equal(
                        got, oracle.batch_varlen(segs, so, lens[smp].copy(), phs, 12, 12, oracle.OP_DATA_CALC)))
                for k in knobs:
                    netcsum.tune(k, RESET[k])
        for tag, d in res.items():
            ms = min(d["ms"])
            line = {"layout": name, "buffer": slot, "segment_at": ix, "n": n, "mean_segment_B": round(seg_bytes / n, 1),
                    "form": tag, "ms_passes": [round(x, 4) for x in d["ms"]], "ms": round(ms, 4),
                    "algorithmic_bytes": algo, "GB_per_s_algorithmic": round(algo / ms / 1e6, 1),
                    "frac_of_8TBps": round(algo / ms / 1e6 / 8000, 4), "kernel": d["kernel"]}
            if "parity_sample_ok" in d:
                line["parity_sample_ok"] = d["parity_sample_ok"]
            print(json.dumps(line), flush=True)
        del base, ph, off_d, len_d, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
