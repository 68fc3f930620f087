#!/usr/bin/env python3
"""Packet batches in the layouts a NIC ring really has (GPU box only; DESIGN.md §9 "NIC-ring layouts").

For 1 M datagrams per layout (tools/ring_layouts.py):
  packed     1500-B IPv4/TCP datagrams back to back (stride 1500)
  template   1500-B datagrams in 1520-B slots at +14 (the reference's template pool buffers,
             Cfg/Template/net_dev_cfg.c:146-149), 1506 B present
  nb2k       1500-B datagrams in 2048-B slots at +64, 1984 B present
  ring       40 / 576 / 1500-B datagrams at 7 : 4 : 1 in 1520-B slots at +14, 1506 B present
each as a strided batch (pkt_len = bytes present) under NETCSUM_TUNE_PKT_BOUND 4 (ring plans: the form
and run length the previous batch on the ring sampled on the device, "strided.plan", with the plan the
timed calls ran) and 0 / 1 / 2 / 3 (the
run-stream kernel reading whole spans / live pieces, the parse first / live pieces with piece 0,
/ with the first 4 pieces loaded during the parse; 3 only for dense layouts) at the default run
length and at 8 / 32 datagrams per run, and as an
offset/length batch (per-frame descriptors: the live-piece stream, and the lane-group kernel with
TUNE_KERNEL 2), fused Rx and Tx finalize. Variants interleaved, two passes; median
HIP-event time of 20 launches after a timed warm-up. After the first Tx every Rx flag must read
IP_OK | L4_OK | L4_CHECKED (valid), and the three bounds and both forms must write identical bytes.
One JSON line per (layout, form, op) to stdout."""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

import netcsum  # noqa: E402
import ring_layouts as rl  # noqa: E402


def events_ms(fn, st, reps=20, warm_s=0.15):
    t0, k = time.perf_counter(), 0
    while k < 3 or time.perf_counter() - t0 < warm_s:
        fn()
        k += 1
        if k % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev)


def main():
    n = int(os.environ.get("RING_N", 1 << 20))
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    layouts = [("packed", 1500, 0, None), ("template", 1520, 14, None), ("nb2k", 2048, 64, None),
               ("ring", 1520, 14, "mixed")]
    want = [x for x in sys.argv[1:]] or [x[0] for x in layouts]
    for name, slot, lead, kind in layouts:
        if name not in want:
            continue
        r = rl.mixed_ring(torch, netcsum, dev, n, slot, lead) if kind else rl.uniform_ring(torch, netcsum, dev, n, slot, lead)
        flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        strided = {"stride": slot, "pkt_len": r["present"]}
        desc = {"off": r["off"], "lens": r["lens"]}
        netcsum.tx_finalize_ipv4(r["base"], n, None, stream=st, **strided)
        torch.cuda.synchronize()
        ref = r["buf"].clone()
        # (tag, bound, datagrams per run, form, pieces in flight); RING_VARIANTS=d8 selects the D=8 set,
        # RING_VARIANTS=runs a sweep of run lengths
        if os.environ.get("RING_VARIANTS") == "d8":
            variants = [("strided.b0", 0, -1, strided, 4), ("strided.b2", 2, -1, strided, 4),
                        ("strided.b2.d8", 2, -1, strided, 8), ("strided.b3.d8", 3, -1, strided, 8),
                        ("strided.b2.s32.d8", 2, 32, strided, 8), ("offlen", -1, -1, desc, 4),
                        ("offlen.d8", -1, -1, desc, 8)]
        elif os.environ.get("RING_VARIANTS") == "runs":                 # run lengths of the default form
            variants = [("strided.b2.s%d" % s, 2, s, strided, 4) for s in (8, 12, 16, 20, 24, 28, 32)]
        elif os.environ.get("RING_VARIANTS") == "offlengrid":           # offset/length runs x residency
            variants = [("offlen.s%d.w%d" % (r, wv), -1, r, desc, 4) for r in (8, 16, 32) for wv in (5, 6, 7, 8)]
            variants += [("strided.plan.w%d" % wv, 4, -1, strided, 4) for wv in (5, 6, 7, 8)]
        elif os.environ.get("RING_VARIANTS") == "offlen":               # offset/length forms only
            variants = [("offlen", -1, -1, desc, 4), ("offlen.s32", -1, 32, desc, 4), ("offlen.s8", -1, 8, desc, 4),
                        ("offlen.w5", -1, -1, desc, 4), ("offlen.w6", -1, -1, desc, 4), ("offlen.s32.w6", -1, 32, desc, 4)]
        elif os.environ.get("RING_VARIANTS") == "plan":                 # the device plan against fixed forms
            variants = [("strided.plan", 4, -1, strided, 4), ("strided.b0", 0, -1, strided, 4),
                        ("strided.b2", 2, -1, strided, 4), ("strided.b2.s8", 2, 8, strided, 4),
                        ("strided.b2.s32", 2, 32, strided, 4), ("offlen", -1, -1, desc, 4),
                        ("offlen.b2.s32", 2, 32, desc, 4)]
        else:
            variants = [("strided.plan", 4, -1, strided, 4),
                        ("strided.b0", 0, -1, strided, 4), ("strided.b1", 1, -1, strided, 4),
                        ("strided.b2", 2, -1, strided, 4), ("strided.b3", 3, -1, strided, 4),
                        ("strided.b2.s8", 2, 8, strided, 4), ("strided.b3.s8", 3, 8, strided, 4),
                        ("strided.b2.s32", 2, 32, strided, 4), ("offlen", -1, -1, desc, 4),
                        ("offlen.b2.s32", 2, 32, desc, 4), ("offlen.lanegroup", -1, -2, desc, 4)]
        res = {}
        for p in range(2):
            for tag, bound, spw, kw, dd in variants:
                netcsum.tune(netcsum.TUNE_CHUNKS, 8 if dd == 8 else 0)
                netcsum.tune(netcsum.TUNE_PKT_BOUND, bound)
                netcsum.tune(netcsum.TUNE_TILE, max(spw, -1))
                netcsum.tune(netcsum.TUNE_KERNEL, 2 if spw == -2 else 0)   # the lane-group packet kernel
                # ".wN": N waves per SIMD resident (TUNE_STREAM_WAVES; default: as many as fit)
                netcsum.tune(netcsum.TUNE_STREAM_WAVES, int(tag.rsplit(".w", 1)[1]) if ".w" in tag else -1)
                base = r["buf"] if kw is desc else r["base"]
                for op in ("rx", "tx"):
                    if op == "rx":
                        flags.zero_()
                        fn = lambda: netcsum.rx_validate_ipv4(base, n, flags, stream=st, **kw)  # noqa: E731
                    else:
                        fn = lambda: netcsum.tx_finalize_ipv4(base, n, None, stream=st, **kw)  # noqa: E731
                    ms = events_ms(fn, st)
                    d = res.setdefault((tag, op), {"ms": [], "kernel": netcsum.last_launch()})
                    d["ms"].append(ms)
                    if bound == 4:                                         # the ring plan the timed calls ran
                        d["plan"] = netcsum.last_launch().rsplit("pkts_per_wave=", 1)[-1]
                    if op == "rx":
                        d["all_valid"] = bool(((flags & 0x07) == 0x07).all().item())
                    else:
                        d["bytes_equal_first_tx"] = bool(torch.equal(r["buf"], ref))
        netcsum.tune(netcsum.TUNE_PKT_BOUND, -1)
        netcsum.tune(netcsum.TUNE_TILE, -1)
        netcsum.tune(netcsum.TUNE_KERNEL, 0)
        netcsum.tune(netcsum.TUNE_CHUNKS, 0)
        netcsum.tune(netcsum.TUNE_STREAM_WAVES, -1)
        for (tag, op), d in res.items():
            algo = r["datagram_bytes"] + n * (1 if op == "rx" else 4)
            ms = min(d["ms"])
            line = {"layout": name, "slot": slot, "ip_header_at": lead, "present": r["present"], "n": n,
                    "mean_datagram_B": round(r["datagram_bytes"] / n, 1), "form": tag, "op": op,
                    "ms_passes": [round(x, 4) for x in d["ms"]], "ms": round(ms, 4),
                    "Mframes_per_s": round(n / ms / 1e3, 1), "algorithmic_bytes": algo,
                    "GB_per_s_algorithmic": round(algo / ms / 1e6, 1),
                    "frac_of_8TBps": round(algo / ms / 1e6 / 8000, 4), "kernel": d["kernel"]}
            line.update({k: v for k, v in d.items() if k not in ("ms", "kernel")})
            print(json.dumps(line), flush=True)
        del r, ref, flags
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
