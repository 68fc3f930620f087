#!/usr/bin/env python3
"""Secondary measurements for DESIGN.md (not the bench.py line): configs C3 and C4 with the library's
default launch policy and a CPU baseline beside each (the oracle's C restatement of net_util.c, -O2,
OpenMP over the host CPUs bench.py uses, data first-touched by the workers, on a bounded sample),
the packet batches (fused Rx, Tx on packed and on NET_BUF-shaped buffers, the offload-seam bursts),
the host-memory (PCIe-inclusive) rates of C2, C4 and the bursts, the per-packet drop-in latency, and
the CPU lines of the packet and chain rows (the stack's per-datagram checksum calls in the C
restatement). Every measured batch is spot-checked against the oracle."""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
import oracle  # noqa: E402
from bench import SEED, c2_pseudo_headers, host_cpus  # noqa: E402


def cpu_rate(fn, nbytes, seconds=2.0):
    """GiB/s of fn() over nbytes per call, repeated for `seconds` after one warm call."""
    fn()
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()
        reps += 1
    return round(reps * nbytes / (time.perf_counter() - t0) / 2 ** 30, 3)


def events_ms(fn, st, reps=20, warm=3, warm_s=0.1):
    # warm by time, not count: the first few ms of launches after an idle gap run at lower clocks
    # (profiles/r1_rx_order.jsonl: 0.316 ms cold vs 0.254 ms warm for the same fused-Rx launch)
    t0 = time.perf_counter()
    k = 0
    while k < warm or time.perf_counter() - t0 < warm_s:
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


def packet_cpu_lines(threads):
    """CPU lines of the packet and chain rows: the C restatement's per-datagram sequence
    (Oracle_PktBatch: HdrVerify + DataVerify on Rx, HdrCalc + DataCalc written on Tx) over a 256 Ki x
    1500-B sample of the same datagrams (IPv4/TCP, IPv6/TCP, alternating), and the per-chain
    DataCalc over 2 Ki of the 64 KiB chains; data first-touched by the OpenMP workers, GiB/s of
    datagram / payload bytes, all host threads and one."""
    ns, L = 1 << 18, 1500
    buf = oracle.fill_parallel(0, ns * L, SEED, 0, n_threads=threads, unit=L)
    v = buf.reshape(ns, L)
    h4 = np.array([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], np.uint8)
    h6 = np.array([0x60, 0, 0, 0, (L - 40) >> 8, (L - 40) & 0xFF, 6, 64], np.uint8)
    res = {"threads": threads, "kind": "port (oracle/net_util_oracle.c -O2: the stack's per-datagram checksum "
           "calls, Oracle_PktBatch / Oracle_BatchChains)", "sample": f"{ns} x {L}-B datagrams (393 MB), "
           "first-touched by the workers; chains: 2048 x 45 fragments"}
    for tag, setup in (("ipv4", lambda: v.__setitem__((slice(None), slice(0, 12)), h4)),
                       ("ipv6", lambda: v.__setitem__((slice(None), slice(0, 8)), h6)),
                       ("mixed", lambda: (v.__setitem__((slice(None), slice(0, 8)), h6),
                                          v.__setitem__((slice(0, None, 2), slice(0, 12)), h4)))):
        setup()
        oracle.pkt_batch(buf, L, L, ns, True, n_threads=threads)             # valid checksums
        ok = bool((oracle.pkt_batch(buf, L, L, ns, False, n_threads=threads) == 7).all())
        for t in (threads, 1):
            sfx = "" if t > 1 else "_1thread"
            res[f"{tag}_rx_GiB_per_s{sfx}"] = cpu_rate(lambda: oracle.pkt_batch(buf, L, L, ns, False, n_threads=t),
                                                      ns * L, seconds=2.0 if t > 1 else 1.0)
            res[f"{tag}_tx_GiB_per_s{sfx}"] = cpu_rate(lambda: oracle.pkt_batch(buf, L, L, ns, True, n_threads=t),
                                                      ns * L, seconds=2.0 if t > 1 else 1.0)
        res[f"{tag}_all_valid"] = ok
    del buf, v
    # the NIC ring of tools/ring_layouts.py: 40 / 576 / 1500-B datagrams (7:4:1) in 1520-B slots, the
    # IPv4 header at +14, 1506 B present per slot; frames per second and GiB/s of datagram bytes
    import ring_layouts as rl
    nr, slot, lead = 1 << 18, 1520, 14
    rbuf = oracle.fill_parallel(0, nr * slot, SEED, 0, n_threads=threads, unit=slot)
    sizes = rl.ring_sizes(nr)
    rbuf.reshape(nr, slot)[:, lead:lead + 40] = rl.headers(sizes)
    rb = rbuf[lead:]
    oracle.pkt_batch(rb, slot, slot - lead, nr, True, n_threads=threads)      # valid checksums
    ok = bool((oracle.pkt_batch(rb, slot, slot - lead, nr, False, n_threads=threads) & 7 == 7).all())
    dgram = int(sizes.sum())
    for t in (threads, 1):
        sfx = "" if t > 1 else "_1thread"
        g = cpu_rate(lambda: oracle.pkt_batch(rb, slot, slot - lead, nr, False, n_threads=t), dgram,
                     seconds=2.0 if t > 1 else 1.0)
        res["ring_rx_GiB_per_s" + sfx] = g
        res["ring_rx_Mframes_per_s" + sfx] = round(g * 2 ** 30 / (dgram / nr) / 1e6, 1)
    res["ring_all_valid"] = ok
    res["ring_sample"] = f"{nr} frames of the 40/576/1500-B ring in 1520-B slots ({dgram / 1e6:.0f} MB of datagrams)"
    del rbuf, rb
    nc, per, B = 1 << 11, 45, 2048
    plen = np.full(per, 1480, np.uint16)
    plen[-1] = 65515 - 1480 * (per - 1) - 8
    lens = np.tile(plen, nc)
    offs = (np.arange(nc * per, dtype=np.uint64) * B + 42).astype(np.uint64)
    first = (np.arange(nc + 1, dtype=np.uint64) * per).astype(np.uint32)
    cb = oracle.fill_parallel(0, nc * per * B, SEED, 0, n_threads=threads, unit=per * B)
    ph = np.zeros((nc, 12), np.uint8)
    ph[:, 9] = 17
    ph = ph.reshape(-1)
    pay = int(lens.astype(np.int64).sum()) + 12 * nc
    for t in (threads, 1):
        res["chains_GiB_per_s" + ("" if t > 1 else "_1thread")] = cpu_rate(
            lambda: oracle.batch_chains(cb, offs, lens, first, ph, 12, 12, nc, 0, n_threads=t), pay,
            seconds=2.0 if t > 1 else 1.0)
    return res


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    out = {}
    # ---- C3: 16 M x 20 B IPv4 headers, HdrCalc
    nh = 1 << 24
    hdr = torch.empty(nh * 20 + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(hdr, nh * 20, SEED, 0)
    o3 = torch.empty(nh, dtype=torch.int16, device=dev)
    ms = events_ms(lambda: netcsum.batch_strided(hdr, 20, 20, None, 0, 0, nh, o3, netcsum.OP_HDR_CALC, stream=st), st)
    idx = np.random.default_rng(0).choice(nh, 512, replace=False)
    host = hdr[: nh * 20].view(nh, 20)[torch.from_numpy(idx).to(dev)].cpu().numpy().reshape(-1)
    ok = np.array_equal(o3.cpu().numpy().view(np.uint16)[idx], oracle.batch_strided(host, 20, 20, None, 0, 0, 512, 2))
    out["C3"] = {"headers": nh, "ms": round(ms, 4), "Ghdr_per_s": round(nh / ms / 1e6, 2), "kernel": netcsum.last_launch(),
                 "GiB_per_s_checksummed": round(nh * 20 / ms / 1e6 / 1.073741824, 1),
                 "GB_per_s_algorithmic": round(nh * 22 / ms / 1e6, 1), "parity_sample_ok": ok}
    threads, _ = host_cpus()
    ns = 1 << 22                                     # 4 Mi headers = 84 MB sample of the C3 shape
    hs = oracle.fill_parallel(0, ns * 20, SEED, 0, n_threads=threads, unit=20)
    for t in (threads, 1):
        g = cpu_rate(lambda: oracle.batch_strided(hs, 20, 20, None, 0, 0, ns, 2, n_threads=t), ns * 20,
                     2.0 if t > 1 else 0.5)
        out["C3"]["cpu_GiB_per_s" + ("" if t > 1 else "_1thread")] = g
    out["C3"]["cpu"] = {"threads": threads, "kind": "port (oracle/net_util_oracle.c -O2, HdrCalc per header)",
                        "sample": f"{ns} x 20-B headers, first-touched by the workers",
                        "Ghdr_per_s": round(out["C3"]["cpu_GiB_per_s"] * 2 ** 30 / 20 / 1e9, 3)}
    del hdr, o3, hs
    torch.cuda.empty_cache()
    # ---- C4: 1 M packed UDP datagrams, 40..9000 B (seed 7), 12-B pseudo each
    rng = np.random.default_rng(7)
    nv = 1 << 20
    lens = rng.integers(40, 9001, size=nv).astype(np.uint16)
    off = np.zeros(nv, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    tot = int(off[-1]) + int(lens[-1])
    base = torch.empty(tot + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(base, tot, SEED, 0)
    ph = np.zeros((nv, 12), np.uint8)
    ph[:, 9] = 17
    ph[:, 10] = (lens >> 8).astype(np.uint8)
    ph[:, 11] = (lens & 0xFF).astype(np.uint8)
    ph_d = torch.from_numpy(ph.reshape(-1)).to(dev)
    off_d = torch.from_numpy(off.view(np.int64)).to(dev)
    len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
    o4 = torch.empty(nv, dtype=torch.int16, device=dev)
    ms = events_ms(lambda: netcsum.batch_varlen(base, off_d, len_d, ph_d, 12, 12, nv, o4, 0, stream=st), st)
    sel = np.arange(0, nv, nv // 256)
    got = o4.cpu().numpy().view(np.uint16)[sel]
    bh = base.cpu().numpy()
    want = oracle.batch_varlen(bh, off[sel], lens[sel], ph[sel].reshape(-1), 12, 12, 0)
    out["C4"] = {"datagrams": nv, "bytes": tot, "odd_starts": int((off & 1).sum()), "ms": round(ms, 4),
                 "GiB_per_s_checksummed": round((tot + 12 * nv) / ms / 1e6 / 1.073741824, 1),
                 "GB_per_s_algorithmic": round((tot + 14 * nv) / ms / 1e6, 1),
                 "descriptor_bytes_per_launch": 10 * nv, "kernel": netcsum.last_launch(), "parity_sample_ok": bool(np.array_equal(got, want))}
    # host-memory C4 (PCIe-inclusive): the same packed datagrams from pinned memory, pipelined
    bh_p = torch.from_numpy(bh[:tot]).pin_memory()
    off_h, len_h = torch.from_numpy(off.view(np.int64)).pin_memory(), torch.from_numpy(lens.view(np.int16)).pin_memory()
    ph_h = torch.from_numpy(ph.reshape(-1)).pin_memory()
    o4h = torch.empty(nv, dtype=torch.int16).pin_memory()
    rates = {}
    for chunks in (4, 16, 64):
        netcsum.batch_varlen_host(bh_p, off_h, len_h, ph_h, 12, 12, nv, o4h, 0, n_chunks=chunks)
        ts = []
        for _ in range(4):
            t0 = time.perf_counter()
            netcsum.batch_varlen_host(bh_p, off_h, len_h, ph_h, 12, 12, nv, o4h, 0, n_chunks=chunks)
            ts.append(time.perf_counter() - t0)
        rates[chunks] = round((tot + 12 * nv) / statistics.median(ts) / 2 ** 30, 2)
    out["C4"]["host_memory_GiB_per_s_by_chunks"] = rates
    out["C4"]["host_memory_parity_ok"] = bool(np.array_equal(o4h.numpy().view(np.uint16)[sel], want))
    del bh_p, off_h, len_h, ph_h, o4h
    # CPU baseline on a 256 Ki-datagram sample of the same length distribution
    threads, _ = host_cpus()
    ncs = 1 << 18
    tot_s = int(off[ncs - 1]) + int(lens[ncs - 1])
    bs = oracle.fill_parallel(0, tot_s, SEED, 0, n_threads=threads, unit=max(1, tot_s // threads))
    for t in (threads, 1):
        g = cpu_rate(lambda: oracle.batch_varlen(bs, off[:ncs], lens[:ncs], ph[:ncs].reshape(-1), 12, 12, 0,
                                                 n_threads=t), tot_s + 12 * ncs, 2.0 if t > 1 else 0.5)
        out["C4"]["cpu_GiB_per_s" + ("" if t > 1 else "_1thread")] = g
    out["C4"]["cpu"] = {"threads": threads, "kind": "port (oracle/net_util_oracle.c -O2, DataCalc per datagram)",
                        "sample": f"first {ncs} datagrams ({tot_s / 1e9:.2f} GB), first-touched by the workers"}
    del base, o4, bh, bs
    torch.cuda.empty_cache()
    # ---- fused Rx validation of 1 M x 1500-B IPv4/TCP datagrams vs the two-pass form
    n, L = 1 << 20, 1500
    pk = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(pk, n * L, SEED, 0)
    v = pk[: n * L].view(n, L)
    hdr = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
    v[:, 0:12] = hdr
    tcp_ph = torch.zeros(n, 12, dtype=torch.uint8, device=dev)
    tcp_ph[:, 0:8] = v[:, 12:20]
    tcp_ph[:, 9] = 6
    tcp_ph[:, 10] = (L - 20) >> 8
    tcp_ph[:, 11] = (L - 20) & 0xFF
    tcp_ph = tcp_ph.reshape(-1).contiguous()
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    netcsum.tx_finalize_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st)      # valid checksums
    torch.cuda.synchronize()
    ms_fused = events_ms(lambda: netcsum.rx_validate_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st), st)
    fused_kernel = netcsum.last_launch()
    ok_all = bool(((flags & 0x07) == 0x07).all().item())
    o_ip = torch.zeros(n, dtype=torch.uint8, device=dev)
    o_l4 = torch.zeros(n, dtype=torch.uint8, device=dev)

    def two_pass():
        netcsum.batch_strided(pk, L, 20, None, 0, 0, n, o_ip, netcsum.OP_HDR_VERIFY, stream=st)
        netcsum.batch_strided(pk.data_ptr() + 20, L, L - 20, tcp_ph, 12, 12, n, o_l4, netcsum.OP_DATA_VERIFY,
                              stream=st)
    ms_two = events_ms(two_pass, st)
    two_ok = bool(o_ip.all().item() and o_l4.all().item())
    out["rx_fused_1500B_tcp"] = {"packets": n, "ms_fused": round(ms_fused, 4), "ms_two_pass": round(ms_two, 4),
                                 "GiB_per_s_fused": round(n * L / ms_fused / 1e6 / 1.073741824, 1),
                                 "GiB_per_s_two_pass": round(n * L / ms_two / 1e6 / 1.073741824, 1),
                                 "all_valid_fused": ok_all, "all_valid_two_pass": two_ok, "kernel": fused_kernel}
    ms_tx = events_ms(lambda: netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st), st)
    out["tx_finalize_1500B_tcp"] = {"ms": round(ms_tx, 4), "GiB_per_s": round(n * L / ms_tx / 1e6 / 1.073741824, 1),
                                    "GB_per_s_algorithmic": round(n * (L + 4) / ms_tx / 1e6, 1),
                                    "kernel": netcsum.last_launch()}
    # NET_BUF-shaped buffers, one per datagram: the reference's template (Cfg/Template/net_dev_cfg.c:
    # 146-149: 1518-B large buffers, 4-B alignment -> 1520-B stride, the datagram after a 14-B Ethernet
    # header, 1506 B present) and 2048-B buffers with the IPv4 header at +64 (both checksum fields in
    # one 64-B line); tools/run_config.py tx_nb / rx_nb / tx_nb2k / rx_nb2k
    out["netbuf_1500B_tcp"] = {}
    for tag, S, lead in (("template_1520", 1520, 14), ("2KiB_at64", 2048, 64)):
        present = S - lead
        nbuf = torch.empty(n * S + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(nbuf, n * S, SEED, 0)
        nv_ = nbuf[: n * S].view(n, S)
        nv_[:, lead:lead + 12] = hdr
        nb = nbuf[lead:]
        netcsum.tx_finalize_ipv4(nb, n, None, stride=S, pkt_len=present, stream=st)
        ms_nb_tx = events_ms(lambda: netcsum.tx_finalize_ipv4(nb, n, None, stride=S, pkt_len=present, stream=st), st)
        k_nb_tx = netcsum.last_launch()
        ms_nb_rx = events_ms(lambda: netcsum.rx_validate_ipv4(nb, n, flags, stride=S, pkt_len=present, stream=st), st)
        out["netbuf_1500B_tcp"][tag] = {
            "stride": S, "ip_header_at": lead, "bytes_present": present,
            "ms_tx": round(ms_nb_tx, 4), "GB_per_s_algorithmic_tx": round(n * (L + 4) / ms_nb_tx / 1e6, 1),
            "ms_rx": round(ms_nb_rx, 4), "GB_per_s_algorithmic_rx": round(n * (L + 1) / ms_nb_rx / 1e6, 1),
            "all_valid_rx": bool(((flags & 0x07) == 0x07).all().item()), "kernel_tx": k_nb_tx,
            "kernel_rx": netcsum.last_launch()}
        del nbuf, nv_, nb
    # ---- the same 1 M x 1500-B datagrams as IPv6/TCP (40-B header, 40-B pseudo-header)
    hdr6 = torch.tensor([0x60, 0, 0, 0, (L - 40) >> 8, (L - 40) & 0xFF, 6, 64], dtype=torch.uint8, device=dev)
    v[:, 0:8] = hdr6
    netcsum.tx_finalize_ipv6(pk, n, flags, stride=L, pkt_len=L, stream=st)
    torch.cuda.synchronize()
    ms6 = events_ms(lambda: netcsum.rx_validate_ipv6(pk, n, flags, stride=L, pkt_len=L, stream=st), st)
    k6 = netcsum.last_launch()
    ok6 = bool(((flags & 0x07) == 0x07).all().item())
    ms6_tx = events_ms(lambda: netcsum.tx_finalize_ipv6(pk, n, None, stride=L, pkt_len=L, stream=st), st)
    # every other datagram back to IPv4 (its header restored, checksums rewritten): a mixed ring
    v[0::2, 0:12] = hdr
    v[0::2, 12:20] = 0x0A
    netcsum.tx_finalize_ip(pk, n, flags, stride=L, pkt_len=L, stream=st)
    torch.cuda.synchronize()
    msmx = events_ms(lambda: netcsum.rx_validate_ip(pk, n, flags, stride=L, pkt_len=L, stream=st), st)
    okmx = bool(((flags & 0x07) == 0x07).all().item())
    out["mixed_v4_v6_1500B_tcp"] = {"packets": n, "ms_rx": round(msmx, 4), "all_valid_rx": okmx,
                                    "GiB_per_s_rx": round(n * L / msmx / 1e6 / 1.073741824, 1)}
    # the checksum-offload seam's bursts on the same mixed ring (actions instead of / beside flags)
    act = torch.zeros(n, dtype=torch.uint8, device=dev)
    ms_rb = events_ms(lambda: netcsum.rx_burst(pk, n, act, stride=L, pkt_len=L, stream=st), st)
    ok_rb = bool((act == 0).all().item())
    ms_tb = events_ms(lambda: netcsum.tx_burst(pk, n, None, stride=L, pkt_len=L, stream=st), st)
    out["offload_bursts_mixed_1500B"] = {
        "ms_rx_burst": round(ms_rb, 4), "GB_per_s_algorithmic_rx": round(n * (L + 1) / ms_rb / 1e6, 1),
        "all_delivered": ok_rb, "ms_tx_burst": round(ms_tb, 4),
        "GB_per_s_algorithmic_tx": round(n * (L + 4) / ms_tb / 1e6, 1), "kernel_tx": netcsum.last_launch()}
    # ... and from pinned host memory (a NIC ring / socket buffers): PCIe-inclusive
    pk_h = torch.empty(n * L, dtype=torch.uint8).pin_memory()
    pk_h.copy_(pk[: n * L])
    act_h = torch.zeros(n, dtype=torch.uint8).pin_memory()
    rate = {}
    for name, fn in (("rx_burst_host", lambda: netcsum.rx_burst_host(pk_h, n, act_h, stride=L, pkt_len=L, n_chunks=16)),
                     ("tx_burst_host", lambda: netcsum.tx_burst_host(pk_h, n, None, stride=L, pkt_len=L, n_chunks=16))):
        fn()
        ts = []
        for _ in range(4):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        rate[name + "_GiB_per_s"] = round(n * L / statistics.median(ts) / 2 ** 30, 2)
    rate["rx_burst_host_all_delivered"] = bool((act_h == 0).all().item())
    rate["tx_burst_host_bytes_equal_device"] = bool(torch.equal(pk_h.to(dev), pk[: n * L]))
    out["offload_bursts_mixed_1500B"].update(rate)
    del pk_h, act_h
    out["ipv6_1500B_tcp"] = {"packets": n, "ms_rx": round(ms6, 4), "ms_tx": round(ms6_tx, 4),
                             "GiB_per_s_rx": round(n * L / ms6 / 1e6 / 1.073741824, 1),
                             "GiB_per_s_tx": round(n * L / ms6_tx / 1e6 / 1.073741824, 1), "all_valid_rx": ok6,
                             "kernel_rx": k6}
    del pk, v, tcp_ph, flags, o_ip, o_l4
    torch.cuda.empty_cache()
    # ---- batched NET_BUF chains: 16 Ki reassembled 64 KiB UDP datagrams, 45 fragments each, every
    #      fragment's payload in its own 2 KiB buffer at ix 42 (Ethernet + IPv4 + 8 B), 12-B pseudo each
    nc, per, B = 1 << 14, 45, 2048
    plen = np.full(per, 1480, np.uint16)
    plen[-1] = 65515 - 1480 * (per - 1) - 8        # 64 KiB datagram incl. UDP header in fragment 0
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
    res = {}
    for g in (16, 32, 64):
        netcsum.tune(netcsum.TUNE_GROUP_LANES, g)
        res[g] = events_ms(lambda: netcsum.batch_chains(base, off_d, len_d, first_d, ph, 12, 12, nc, oc, 0,
                                                        stream=st, n_pieces=nc * per), st)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, 0)
    ms = events_ms(lambda: netcsum.batch_chains(base, off_d, len_d, first_d, ph, 12, 12, nc, oc, 0, stream=st,
                                                n_pieces=nc * per), st)
    k = 256
    hb = base[: k * per * B + 256].cpu().numpy()
    want = oracle.batch_chains(hb, offs[: k * per], lens[: k * per], first[: k + 1], ph[: 12 * k].cpu().numpy(),
                               12, 12, k, 0)
    payload = int(lens.astype(np.int64).sum())
    out["chains_64KiB_datagrams"] = {
        "chains": nc, "pieces_per_chain": per, "payload_bytes": payload, "ms": round(ms, 4),
        "ms_by_group": {str(g): round(v, 4) for g, v in res.items()},
        "GiB_per_s_checksummed": round((payload + 12 * nc) / ms / 1e6 / 1.073741824, 1),
        "GB_per_s_algorithmic": round((payload + 10 * nc * per + 18 * nc) / ms / 1e6, 1),
        "parity_sample_ok": bool(np.array_equal(oc[:k].cpu().numpy().view(np.uint16), want))}
    del base, off_d, len_d, first_d, oc, hb
    torch.cuda.empty_cache()
    # ---- host-memory (PCIe-inclusive) C2 rate: pinned NIC/socket buffers -> GPU -> pinned results
    n, L = 1 << 20, 1500
    seg_h = torch.empty(n * L, dtype=torch.uint8).pin_memory()
    seg_h.numpy()[:] = oracle.fill(0, n * L, SEED, 0)
    ph_h = torch.from_numpy(c2_pseudo_headers(0, n, L, 12)).pin_memory()
    res_h = torch.empty(n, dtype=torch.int16).pin_memory()
    rates = {}
    for chunks in (1, 4, 16, 64):
        netcsum.batch_strided_host(seg_h, L, L, ph_h, 12, 12, n, res_h, 0, n_chunks=chunks)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            netcsum.batch_strided_host(seg_h, L, L, ph_h, 12, 12, n, res_h, 0, n_chunks=chunks)
            ts.append(time.perf_counter() - t0)
        rates[chunks] = round(n * (L + 12) / statistics.median(ts) / 2 ** 30, 2)
    sel = np.arange(0, n, n // 256)
    want = oracle.batch_strided(seg_h.numpy(), L, L, ph_h.numpy(), 12, 12, n, 0, n_threads=8)
    out["C2_host_memory"] = {"GiB_per_s_by_chunks": rates, "parity_ok": bool(np.array_equal(
        res_h.numpy().view(np.uint16), want)), "note": "pinned host in/out, H2D + kernel + D2H pipelined"}
    # ---- per-packet drop-in latency (C1 shape: 72-B UDP datagram + 12-B pseudo)
    ch = netcsum.Chain([{"data": bytes(range(92)), "proto": netcsum.NET_PROTOCOL_TYPE_UDP_V4, "transport_ix": 20,
                         "transport_hdr_len": 8, "data_len": 64}])
    phb = netcsum.HostBytes(bytes(12))
    for _ in range(50):
        netcsum.DataCalc(ch.ptr, phb.ptr, 12)
    t0 = time.perf_counter()
    for _ in range(2000):
        netcsum.DataCalc(ch.ptr, phb.ptr, 12)
    us = (time.perf_counter() - t0) / 2000 * 1e6
    out["C1_dropin_call_us"] = round(us, 2)
    # ---- CRC-32 (net_util.c:485-636): 1 M x 1500-B frames (16-lane groups) and 16 M 6-B MAC
    #      addresses (one lane each), CalcCpl, device-resident
    nf, Lf = 1 << 20, 1500
    fr = torch.empty(nf * Lf + 64, dtype=torch.uint8, device=dev)
    netcsum.fill(fr, nf * Lf, SEED, 0)
    fo = torch.empty(nf, dtype=torch.int32, device=dev)
    ms_f = events_ms(lambda: netcsum.crc32_strided(fr, Lf, Lf, nf, fo, 1, stream=st), st)
    kf = netcsum.last_launch()
    del fr
    nm = 1 << 24
    macs = torch.empty(nm * 6 + 64, dtype=torch.uint8, device=dev)
    netcsum.fill(macs, nm * 6, SEED, 0)
    mo = torch.empty(nm, dtype=torch.int32, device=dev)
    ms_m = events_ms(lambda: netcsum.crc32_strided(macs, 6, 6, nm, mo, 1, stream=st), st)
    out["crc32"] = {"frames_1500B": {"n": nf, "ms": round(ms_f, 4), "GB_per_s": round(nf * (Lf + 4) / ms_f / 1e6, 1),
                                     "kernel": kf},
                    "macs_6B": {"n": nm, "ms": round(ms_m, 4), "G_per_s": round(nm / ms_m / 1e6, 2),
                                "GB_per_s": round(nm * 10 / ms_m / 1e6, 1), "kernel": netcsum.last_launch()}}
    out["cpu_packet_rows"] = packet_cpu_lines(host_cpus()[0])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
