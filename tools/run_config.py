#!/usr/bin/env python3
"""Run ONE BASELINE config's default launch N times (for rocprofv3 kernel-trace / --pmc passes; GPU
box only). Usage: python tools/run_config.py <c2|c3|c4|c5|rx|tx|tx2> [reps]
  c2  1 M x 1500 B + 12-B pseudo, DataCalc       c3  16 M x 20-B IPv4 headers, HdrCalc
  c2np  C2 without pseudo-headers (diagnostic)
  c4  1 M packed UDP 40-9000 B + pseudo          c5  16 M x 1500 B + pseudo (one GPU's shard)
  rx / tx  fused Rx / Tx finalize, 1 M x 1500-B IPv4/TCP, strided; tx2 = two-pass Tx
  rx6 / rxmix  fused Rx of the same datagrams as IPv6/TCP / alternating IPv4 and IPv6 (bench_configs)
  crc  CRC-32 CalcCpl of 1 M x 1500-B frames, strided (the library's default CRC form)
  tx_nb / rx_nb  Tx finalize / fused Rx on NET_BUF-shaped buffers of the reference's template
       (Cfg/Template/net_dev_cfg.c:146-149: 1518-B large buffers, 4-B alignment -> a 1520-B stride):
       the 1500-B IPv4/TCP datagram after a 14-B Ethernet header, 1506 B present per buffer
  tx_nb2k / rx_nb2k  the same in 2048-B buffers with the IPv4 header at +64 (both checksum fields
       in one 64-B line)
  rx_sNNNN / tx_sNNNN  the 1500-B datagrams at stride NNNN (1500 = packed), 1500 B present
  rxb / txb  the offload-seam bursts (RxBurst / TxBurst) on 1 M x 1500-B alternating IPv4 / IPv6
  rx_ring / tx_ring  1 M mixed 40/576/1500-B datagrams (7:4:1) in 1520-B slots at +14, strided,
       pkt_len 1506; rx_ringv / tx_ringv the same ring by offset/length descriptors; rx_nb2kv /
       tx_nb2kv 1500-B datagrams in 2-KiB slots at +64 by descriptors (tools/ring_layouts.py)
  suffix .bN = NETCSUM_TUNE_PKT_BOUND N, .sN = packets per wave run, .ntN = NETCSUM_TUNE_NT_LOADS N,
  .kN = NETCSUM_TUNE_KERNEL N (chains.k3 / .k4: pass 1 in round 5's live form / tiled groups), .dN = NETCSUM_TUNE_CHUNKS N,
  .xN = NETCSUM_TUNE_STREAM_XCD N, .gN = NETCSUM_TUNE_STORE_GATHER N, .wN = NETCSUM_TUNE_STREAM_WAVES N,
  .cgN = NETCSUM_TUNE_CHAIN_GRID N, .tN = NETCSUM_TUNE_STREAM_TOUCH N, .lcN = NETCSUM_TUNE_LIVE_COMPACT N,
  .ccN = NETCSUM_TUNE_CHAIN_COMBINE N
  (e.g. rx_ring.b0.s32, rx_nb2k.nt0)
  chains  16 Ki NET_BUF chains of 45 fragments (64 KiB UDP datagrams, each fragment in its own
       2 KiB buffer at +42), DataCalc
  pool1520 / pool1520mix / pool2k / pool2kmix  ChkSumBatchVarLen over one segment per pool buffer
       (tools/varlen_pool_probe.py)
Prints the launch description and the mean ms per launch (HIP events), and the algorithmic bytes."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED, c2_pseudo_headers  # noqa: E402


def main():
    name = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    # suffixes: ".bN" = NETCSUM_TUNE_PKT_BOUND N, ".sN" = TUNE_TILE N (packets per wave run),
    # ".ntN" = NETCSUM_TUNE_NT N (NETCSUM_TUNE_NT_LOADS; 0: plain-policy stream loads)
    for part in name.split(".")[1:]:
        if part.startswith("nt"):
            netcsum.tune(netcsum.TUNE_NT_LOADS, int(part[2:]))
            continue
        if part[:2] == "cc":
            netcsum.tune(netcsum.TUNE_CHAIN_COMBINE, int(part[2:]))
            continue
        if part[:2] == "lc":
            netcsum.tune(netcsum.TUNE_LIVE_COMPACT, int(part[2:]))
            continue
        if part[:1] == "t":
            netcsum.tune(netcsum.TUNE_STREAM_TOUCH, int(part[1:]))
        elif part[:1] == "d":
            netcsum.tune(netcsum.TUNE_CHUNKS, int(part[1:]))
        elif part[:1] == "k":
            netcsum.tune(netcsum.TUNE_KERNEL, int(part[1:]))
        elif part[:1] == "b":
            netcsum.tune(netcsum.TUNE_PKT_BOUND, int(part[1:]))
        elif part[:1] == "s":
            netcsum.tune(netcsum.TUNE_TILE, int(part[1:]))
        elif part[:1] == "w":
            netcsum.tune(netcsum.TUNE_STREAM_WAVES, int(part[1:]))
        elif part[:1] == "x":
            netcsum.tune(netcsum.TUNE_STREAM_XCD, int(part[1:]))
        elif part[:2] == "cg":
            netcsum.tune(netcsum.TUNE_CHAIN_GRID, int(part[2:]))
        elif part[:1] == "g":
            netcsum.tune(netcsum.TUNE_STORE_GATHER, int(part[1:]))
    name = name.split(".")[0]
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    if name in ("rx_ring", "tx_ring", "rx_ringv", "tx_ringv", "rx_nb2kv", "tx_nb2kv"):
        # the NIC-ring layouts of tools/ring_layouts.py: mixed 40/576/1500-B datagrams in 1520-B
        # slots at +14 (ring) or 1500-B datagrams in 2-KiB slots at +64 (nb2k); strided with the
        # slot's present bytes as pkt_len, or "v": offset/length descriptors (frame length - 14)
        import ring_layouts as rl
        n = 1 << 20
        r = (rl.mixed_ring(torch, netcsum, dev, n) if "ring" in name else rl.uniform_ring(torch, netcsum, dev, n, 2048, 64))
        flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        kw = ({"off": r["off"], "lens": r["lens"]} if name.endswith("v") else {"stride": r["slot"], "pkt_len": r["present"]})
        base = r["buf"] if name.endswith("v") else r["base"]
        netcsum.tx_finalize_ipv4(base, n, None, stream=st, **kw)
        if name.startswith("tx"):
            fn = lambda: netcsum.tx_finalize_ipv4(base, n, None, stream=st, **kw)  # noqa: E731
            algo = r["datagram_bytes"] + 4 * n
        else:
            fn = lambda: netcsum.rx_validate_ipv4(base, n, flags, stream=st, **kw)  # noqa: E731
            algo = r["datagram_bytes"] + n
    elif name in ("c2", "c5", "c2np"):
        # c2np: C2 without its pseudo-header stream (a diagnostic, not a BASELINE config)
        n, L = (1 << 24) if name == "c5" else (1 << 20), 1500
        seg = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(seg, n * L, SEED, 0)
        ph = torch.from_numpy(c2_pseudo_headers(0, n, L, 12)).to(dev) if name != "c2np" else None
        pl = 0 if ph is None else 12
        out = torch.empty(n, dtype=torch.int16, device=dev)
        fn = lambda: netcsum.batch_strided(seg, L, L, ph, pl, pl, n, out, 0, stream=st)  # noqa: E731
        algo = n * (L + pl + 2)
    elif name == "c3":
        n, L = 1 << 24, 20
        hdr = torch.empty(n * L, dtype=torch.uint8, device=dev)
        netcsum.fill(hdr, n * L, SEED, 0)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        fn = lambda: netcsum.batch_strided(hdr, L, L, None, 0, 0, n, out, 2, stream=st)  # noqa: E731
        algo = n * (L + 2)
    elif name == "crc":
        n, L = 1 << 20, 1500
        fr = torch.empty(n * L + 64, dtype=torch.uint8, device=dev)
        netcsum.fill(fr, n * L, SEED, 0)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        fn = lambda: netcsum.crc32_strided(fr, L, L, n, out, 1, stream=st)  # noqa: E731
        algo = n * (L + 4)
    elif name == "c4":
        n = 1 << 20
        lens = np.random.default_rng(7).integers(40, 9001, size=n).astype(np.uint16)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        total = int(off[-1]) + int(lens[-1])
        base = torch.empty(total + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(base, total, SEED, 0)
        off_d = torch.from_numpy(off.view(np.int64)).to(dev)
        len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
        ph = torch.from_numpy(np.random.default_rng(1).integers(0, 256, size=12 * n, dtype=np.uint8)).to(dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        fn = lambda: netcsum.batch_varlen(base, off_d, len_d, ph, 12, 12, n, out, 0, stream=st)  # noqa: E731
        algo = total + 12 * n + 2 * n
    elif name.startswith("pool"):
        # ChkSumBatchVarLen over one TCP segment per NET_BUF pool buffer (tools/varlen_pool_probe.py's
        # layouts): 1480-B or 20/556/1480-B mix segments at +34 of 1520-B / +84 of 2048-B buffers
        from varlen_pool_probe import LAYOUTS
        slot, ix, mix = LAYOUTS[name]
        n = 1 << 20
        rng = np.random.default_rng(5)
        lens = (np.array([20, 556, 1480])[rng.choice(3, size=n, p=[7 / 12, 4 / 12, 1 / 12])] if mix
                else np.full(n, 1480)).astype(np.uint16)
        offs = (np.arange(n, dtype=np.uint64) * np.uint64(slot) + np.uint64(ix)).astype(np.uint64)
        base = torch.empty(n * slot + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(base, n * slot, SEED, 0)
        ph = torch.from_numpy(rng.integers(0, 256, size=n * 12, dtype=np.uint8)).to(dev)
        off_d = torch.from_numpy(offs.view(np.int64)).to(dev)
        len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        fn = lambda: netcsum.batch_varlen(base, off_d, len_d, ph, 12, 12, n, out, 0, stream=st)  # noqa: E731
        algo = int(lens.astype(np.int64).sum()) + 14 * n
    elif name == "chains":
        nc, per, B = 1 << 14, 45, 2048
        plen = np.full(per, 1480, np.uint16)
        plen[-1] = 65515 - 1480 * (per - 1) - 8
        lens = np.tile(plen, nc)
        offs = (np.arange(nc * per, dtype=np.uint64) * B + 42).astype(np.uint64)
        first = (np.arange(nc + 1, dtype=np.uint64) * per).astype(np.uint32)
        base = torch.empty(nc * per * B + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(base, nc * per * B, SEED, 0)
        ph = torch.zeros(nc * 12, dtype=torch.uint8, device=dev)
        off_d = torch.from_numpy(offs.view(np.int64)).to(dev)
        len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
        first_d = torch.from_numpy(first.view(np.int32)).to(dev)
        out = torch.empty(nc, dtype=torch.int16, device=dev)
        fn = lambda: netcsum.batch_chains(base, off_d, len_d, first_d, ph, 12, 12, nc, out, 0, stream=st,  # noqa: E731
                                          n_pieces=nc * per)
        algo = int(lens.astype(np.int64).sum()) + 12 * nc + 2 * nc
    elif name in ("tx_nb", "rx_nb", "tx_nb2k", "rx_nb2k") or name.startswith(("rx_s", "tx_s")):
        n, L = 1 << 20, 1500
        S, lead = (2048, 64) if name.endswith("2k") else (1520, 14)
        present = min(S - lead, 65535)
        if name.startswith(("rx_s", "tx_s")):                     # rx_sNNNN: stride NNNN, datagram at 0
            S, lead, present = int(name[4:]), 0, 1500
        nbuf = torch.empty(n * S + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(nbuf, n * S, SEED, 0)
        nbuf[: n * S].view(n, S)[:, lead:lead + 12] = torch.tensor(
            [0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
        nb = nbuf[lead:]
        flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        netcsum.tx_finalize_ipv4(nb, n, None, stride=S, pkt_len=present, stream=st)
        if name.startswith("tx"):
            fn = lambda: netcsum.tx_finalize_ipv4(nb, n, None, stride=S, pkt_len=present, stream=st)  # noqa: E731
            algo = n * (L + 4)
        else:
            fn = lambda: netcsum.rx_validate_ipv4(nb, n, flags, stride=S, pkt_len=present, stream=st)  # noqa: E731
            algo = n * (L + 1)
    else:
        n, L = 1 << 20, 1500
        pk = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(pk, n * L, SEED, 0)
        v = pk[: n * L].view(n, L)
        v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8,
                                  device=dev)
        flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        if name == "tx2":
            netcsum.tune(netcsum.TUNE_TX_PASSES, 2)
        if name in ("rx6", "rxmix", "rxb", "txb"):
            v[:, 0:8] = torch.tensor([0x60, 0, 0, 0, (L - 40) >> 8, (L - 40) & 0xFF, 6, 64], dtype=torch.uint8,
                                     device=dev)
            if name in ("rxmix", "rxb", "txb"):
                v[0::2, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0],
                                             dtype=torch.uint8, device=dev)
                v[0::2, 12:20] = 0x0A
            netcsum.tx_finalize_ip(pk, n, flags, stride=L, pkt_len=L, stream=st)
            fn = lambda: netcsum.rx_validate_ip(pk, n, flags, stride=L, pkt_len=L, stream=st)  # noqa: E731
            if name == "rx6":
                fn = lambda: netcsum.rx_validate_ipv6(pk, n, flags, stride=L, pkt_len=L, stream=st)  # noqa: E731
            act = torch.zeros(n, dtype=torch.uint8, device=dev)
            if name == "rxb":
                fn = lambda: netcsum.rx_burst(pk, n, act, stride=L, pkt_len=L, stream=st)  # noqa: E731
            algo = n * (L + 1)
            if name == "txb":
                fn = lambda: netcsum.tx_burst(pk, n, None, stride=L, pkt_len=L, stream=st)  # noqa: E731
                algo = n * (L + 4)
        elif name == "rx":
            fn = lambda: netcsum.rx_validate_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st)  # noqa: E731
            algo = n * (L + 1)
        else:
            fn = lambda: netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st)  # noqa: E731
            algo = n * (L + 4)
    # warm up by time (the first ~100 launches after an idle gap run at lower clocks);
    # pmc_kernels.py averages only the `reps` launches after these
    import time
    warm, t0 = 0, time.perf_counter()
    while warm < 3 or time.perf_counter() - t0 < (0.5 if reps > 5 else 0.0):
        fn()
        warm += 1
        if warm % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"{name} {netcsum.last_launch()} ms={ms:.4f} algo_bytes={algo} GBps={algo / ms / 1e6:.1f} "
          f"warm_launches={warm} reps={reps}", flush=True)


if __name__ == "__main__":
    main()
