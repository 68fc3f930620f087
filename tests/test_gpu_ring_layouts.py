"""GPU parity of the packet batches on NIC-ring layouts, against the packet oracle
(oracle/oracle_packets.py): frames of mixed sizes in fixed-size slots — the reference's pool
buffers (Cfg/Template/net_dev_cfg.c:146-149: 1518-B buffers, 4-B aligned, so 1520-B slots; the
IPv4 header after a 14-B Ethernet header) and 2-KiB slots with the header at +64 — passed either
strided with the slot's present bytes as pkt_len, or by per-frame offset/length descriptors (the
frame length the driver reports, IF/net_if.c:6593, minus the Ethernet header; at least 46 B).

The strided form runs under every NETCSUM_TUNE_PKT_BOUND: 0 reads whole slots, 1-3 only the pieces
and 64-B sectors holding summed bytes (live pieces, dead pieces skipped; 2 and 3 load the run's first
piece / pieces while the parse runs). The bytes a bounded stream
skips are random here, so a kernel that summed any of them would disagree with the oracle; the bytes
outside the checksum fields must come back untouched by Tx."""
import random
import zlib

import numpy as np
import pytest

import netcsum
import oracle_packets as op
from packets import KINDS, KINDS6, make_packet, make_packet_v6

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _defaults():
    def reset():
        netcsum.tune(netcsum.TUNE_PKT_BOUND, -1)
        netcsum.tune(netcsum.TUNE_TILE, -1)
        netcsum.tune(netcsum.TUNE_TX_PASSES, 0)
        netcsum.tune(netcsum.TUNE_CHUNKS, 0)
    reset()
    yield
    reset()


def _frame(rng, v6=False):
    """A datagram of the ring's size mix (ACK-sized / 576 B / full size), or a random kind."""
    r = rng.random()
    if r < 0.45:
        payload = rng.randint(0, 12)
    elif r < 0.75:
        payload = rng.randint(500, 560)
    elif r < 0.85:
        payload = rng.randint(1400, 1460)
    else:
        payload = rng.randint(0, 1460)
    if v6:
        return make_packet_v6(rng, rng.choice(KINDS6), payload=payload)
    kind = rng.choice(KINDS + ["tcp", "tcp", "udp"])
    return make_packet(rng, kind, payload=payload)


def _ring(rng, n, slot, lead, v6mix=False):
    buf = np.frombuffer(rng.randbytes(n * slot + 64), np.uint8).copy()
    lens = np.zeros(n, np.uint16)
    for i in range(n):
        p = _frame(rng, v6=v6mix and rng.random() < 0.5)[: slot - lead]
        o = i * slot + lead
        buf[o:o + len(p)] = np.frombuffer(p, np.uint8)
        lens[i] = max(len(p), 46) if rng.random() < 0.95 else rng.randint(0, len(p))   # a few truncated
    return buf, lens


def _want(buf, n, slot, lead, present, udp_tx_csum, lens=None):
    rx = np.zeros(n, np.uint8)
    tx = buf.copy()
    txf = np.zeros(n, np.uint8)
    for i in range(n):
        o = i * slot + lead
        m = present if lens is None else int(lens[i])
        pkt = bytes(buf[o:o + m])
        rx[i] = op.rx_validate(pkt)
        q, txf[i] = op.tx_finalize(pkt, udp_tx_csum)
        tx[o:o + m] = np.frombuffer(q, np.uint8)
    return rx, tx, txf


def _want_ip(buf, n, slot, lead, present, udp_tx_csum):
    rx = np.zeros(n, np.uint8)
    tx = buf.copy()
    txf = np.zeros(n, np.uint8)
    for i in range(n):
        o = i * slot + lead
        pkt = bytes(buf[o:o + present])
        rx[i] = op.rx_validate_ip(pkt)
        q, txf[i] = op.tx_finalize_ip(pkt, udp_tx_csum)
        tx[o:o + present] = np.frombuffer(q, np.uint8)
    return rx, tx, txf


def _check(got, want, what):
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (what, [(int(i), int(got[i]), int(want[i])) for i in bad[:6]])


@pytest.mark.parametrize("bound", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("slot,lead", [(1520, 14), (2048, 64), (1536, 1), (9216, 2)])
@pytest.mark.parametrize("passes", [1, 2])
def test_strided_ring_every_bound_vs_oracle(bound, slot, lead, passes):
    netcsum.tune(netcsum.TUNE_PKT_BOUND, bound)
    netcsum.tune(netcsum.TUNE_TX_PASSES, passes)
    rng = random.Random(slot * 7 + lead * 3 + bound)
    n, present = (1500 if slot < 4096 else 300), slot - lead
    buf, _ = _ring(rng, n, slot, lead)
    rx_w, tx_w, txf_w = _want(buf, n, slot, lead, present, True)
    b = torch.from_numpy(buf).to(DEV)
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.rx_validate_ipv4(b[lead:], n, f, stride=slot, pkt_len=present)
    torch.cuda.synchronize()
    assert netcsum.last_launch().startswith("pkt_stream_kernel"), netcsum.last_launch()
    _check(f.cpu().numpy(), rx_w, "rx")
    ft = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv4(b[lead:], n, ft, stride=slot, pkt_len=present)
    torch.cuda.synchronize()
    _check(b.cpu().numpy(), tx_w, "tx bytes")
    _check(ft.cpu().numpy(), txf_w, "tx flags")


@pytest.mark.parametrize("bound", [0, 1, 2, 3])
@pytest.mark.parametrize("spw", [1, 8, 64])
def test_mixed_version_ring_every_bound_vs_oracle(bound, spw):
    """IPv4 and IPv6 frames in one 1520-B-slot ring (RxValidateIP / TxFinalizeIP), runs of 1..64."""
    netcsum.tune(netcsum.TUNE_PKT_BOUND, bound)
    netcsum.tune(netcsum.TUNE_TILE, spw)
    rng = random.Random(1000 + 10 * bound + spw)
    n, slot, lead = 900, 1520, 14
    present = slot - lead
    buf, _ = _ring(rng, n, slot, lead, v6mix=True)
    rx_w, tx_w, txf_w = _want_ip(buf, n, slot, lead, present, True)
    b = torch.from_numpy(buf).to(DEV)
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.rx_validate_ip(b[lead:], n, f, stride=slot, pkt_len=present)
    torch.cuda.synchronize()
    _check(f.cpu().numpy(), rx_w, "rx")
    ft = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ip(b[lead:], n, ft, stride=slot, pkt_len=present)
    torch.cuda.synchronize()
    _check(b.cpu().numpy(), tx_w, "tx bytes")
    _check(ft.cpu().numpy(), txf_w, "tx flags")


@pytest.mark.parametrize("slot,lead", [(1520, 14), (2048, 64)])
def test_offset_length_ring_vs_oracle(slot, lead):
    """The same rings by per-frame descriptors: each frame's reported length, some truncated."""
    rng = random.Random(77 + slot)
    n = 1500
    buf, lens = _ring(rng, n, slot, lead)
    rx_w, tx_w, txf_w = _want(buf, n, slot, lead, None, True, lens=lens)
    b = torch.from_numpy(buf).to(DEV)
    off = torch.from_numpy((np.arange(n, dtype=np.int64) * slot + lead)).to(DEV)
    ln = torch.from_numpy(lens.view(np.int16)).to(DEV)
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.rx_validate_ipv4(b, n, f, off=off, lens=ln)
    torch.cuda.synchronize()
    _check(f.cpu().numpy(), rx_w, "rx")
    ft = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv4(b, n, ft, off=off, lens=ln)
    torch.cuda.synchronize()
    _check(b.cpu().numpy(), tx_w, "tx bytes")
    _check(ft.cpu().numpy(), txf_w, "tx flags")


def test_bounded_stream_full_size_ring_properties():
    """1 M frames of the 40/576/1500-B mix in 1520-B slots (the probe's ring, tools/ring_layouts.py
    shape, built here): Tx under every bound writes the same bytes, then every frame verifies; a
    corrupted byte inside a datagram is caught, one in a slot's unused tail is not read."""
    n, slot, lead = 1 << 20, 1520, 14
    rng = np.random.default_rng(3)
    sizes = np.array([40, 576, 1500])[rng.choice(3, size=n, p=[7 / 12, 4 / 12, 1 / 12])]
    b = torch.randint(0, 256, (n * slot + 64,), dtype=torch.uint8, device=DEV)
    h = rng.integers(0, 256, size=(n, 40), dtype=np.uint8)
    udp = sizes == 576
    h[:, 0], h[:, 1], h[:, 2], h[:, 3] = 0x45, 0, sizes >> 8, sizes & 0xFF
    h[:, 6], h[:, 7], h[:, 9], h[:, 10], h[:, 11] = 0x40, 0, np.where(udp, 17, 6), 0, 0
    h[:, 32] = np.where(udp, h[:, 32], 0x50)
    h[:, 24], h[:, 25] = np.where(udp, (sizes - 20) >> 8, h[:, 24]), np.where(udp, (sizes - 20) & 0xFF, h[:, 25])
    b[: n * slot].view(n, slot)[:, lead:lead + 40] = torch.from_numpy(h).to(DEV)
    base = b[lead:]
    outs = []
    for bound in (0, 1, 2, 3):
        netcsum.tune(netcsum.TUNE_PKT_BOUND, bound)
        c = b.clone()
        netcsum.tx_finalize_ipv4(c[lead:], n, None, stride=slot, pkt_len=slot - lead)
        outs.append(c)
    torch.cuda.synchronize()
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    b.copy_(outs[2])
    del outs
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tune(netcsum.TUNE_PKT_BOUND, -1)
    netcsum.rx_validate_ipv4(base, n, f, stride=slot, pkt_len=slot - lead)
    torch.cuda.synchronize()
    assert bool(((f & 0x07) == 0x07).all().item())
    # corrupt one payload byte inside datagram k, and one byte past the end of datagram j
    k, j = 12345, int(np.nonzero(sizes == 40)[0][100])
    bv = b[: n * slot].view(n, slot)
    bv[k, lead + int(sizes[k]) - 1] ^= 0x5A
    bv[j, lead + 60] ^= 0xA5
    netcsum.rx_validate_ipv4(base, n, f, stride=slot, pkt_len=slot - lead)
    torch.cuda.synchronize()
    fl = f.cpu().numpy()
    assert (fl[k] & 0x07) == 0x05                                # L4 checked, not OK
    assert (np.delete(fl, k) & 0x07 == 0x07).all()


@pytest.mark.parametrize("order", ["sorted", "reversed", "shuffled", "duplicates", "far", "packed", "pairs"])
@pytest.mark.parametrize("spw", [-1, 1, 7, 32, 64])
@pytest.mark.parametrize("bound", [1, 2, 4])
def test_offset_length_runs_every_order_vs_oracle(order, spw, bound):
    """Offset/length batches in the live-piece stream (netcsum_pktstream.hip, VL): a run of
    descriptors in increasing address order within the bitmap's reach streams; any other run (reversed
    or shuffled rings, the same datagram listed twice, slots > 128 KiB apart, neighbours swapped, runs
    of 32 / 64 slots that outgrow the 63-KiB reach) is listed for the deferred pass, which streams it in
    ordered sub-runs inside the reach (a datagram out of order: a sub-run of one). Bound 4: ring plans
    (the plan block samples the descriptors; run length and residency for the next batch). Mixed IPv4 /
    IPv6 (RxValidateIP, TxFinalizeIP, RxBurst), 1520-B slots (2-KiB slots for runs of 32), results
    equal the oracle's; each batch twice (the second in the plan)."""
    netcsum.tune(netcsum.TUNE_TILE, spw)
    netcsum.tune(netcsum.TUNE_PKT_BOUND, bound)
    rng = random.Random(zlib.crc32(f"{order}/{spw}".encode()))
    n, slot, lead = 700, (2048 if spw == 32 else 1520), 14
    buf, lens = _ring(rng, n, slot, lead, v6mix=True)
    offs = np.arange(n, dtype=np.int64) * slot + lead
    if order == "pairs":                                          # neighbours 3 <-> 4 of every 10 swapped
        i = np.arange(3, n - 1, 10)
        offs[i], offs[i + 1] = offs[i + 1].copy(), offs[i].copy()
        lens[i], lens[i + 1] = lens[i + 1].copy(), lens[i].copy()
    if order == "reversed":
        offs, lens = offs[::-1].copy(), lens[::-1].copy()
    elif order == "shuffled":
        perm = np.random.default_rng(spw + 5).permutation(n)
        offs, lens = offs[perm].copy(), lens[perm].copy()
    elif order == "duplicates":
        offs[1::9] = offs[0::9][: len(offs[1::9])]
        lens[1::9] = lens[0::9][: len(lens[1::9])]
    elif order == "far":                                          # every 5th slot 200 KiB further on
        big = np.frombuffer(rng.randbytes(len(buf) + (n // 5 + 1) * 200 * 1024), np.uint8).copy()
        shift = (np.arange(n) // 5) * 200 * 1024
        for i in range(n):
            big[offs[i] + shift[i] - lead:offs[i] + shift[i] - lead + slot] = buf[i * slot:(i + 1) * slot]
        buf, offs = big, offs + shift
    elif order == "packed":                                       # back to back, odd starts, no gaps
        frames = [bytes(buf[o:o + int(m)]) for o, m in zip(offs.tolist(), lens.tolist())]
        pos, parts, new = 1, [b"\x00"], []
        for f in frames:
            new.append(pos)
            parts.append(f)
            pos += len(f)
        buf = np.frombuffer(b"".join(parts) + rng.randbytes(64), np.uint8).copy()
        offs = np.array(new, np.int64)
    frames = [bytes(buf[o:o + int(m)]) for o, m in zip(offs.tolist(), lens.tolist())]
    want_f = np.array([op.rx_validate_ip(f) for f in frames], np.uint8)
    b = torch.from_numpy(buf).to(DEV)
    o_d = torch.from_numpy(offs).to(DEV)
    l_d = torch.from_numpy(lens.view(np.int16)).to(DEV)
    for _ in range(2 if bound == 4 else 1):
        f = torch.zeros(n, dtype=torch.uint8, device=DEV)
        netcsum.rx_validate_ip(b, n, f, off=o_d, lens=l_d)
        torch.cuda.synchronize()
        assert netcsum.last_launch().startswith("pkt_stream_kernel") and "offlen" in netcsum.last_launch()
        _check(f.cpu().numpy(), want_f, "rx")
    if order == "duplicates":
        return                                                    # Tx of one datagram twice: a race by contract
    tx_w = buf.copy()
    txf_w = np.zeros(n, np.uint8)
    for i, (o, m) in enumerate(zip(offs.tolist(), lens.tolist())):
        q, txf_w[i] = op.tx_finalize_ip(bytes(buf[o:o + int(m)]), True)
        tx_w[o:o + int(m)] = np.frombuffer(q, np.uint8)
    for passes in (1, 2):
        netcsum.tune(netcsum.TUNE_TX_PASSES, passes)
        bt = torch.from_numpy(buf).to(DEV)
        ft = torch.zeros(n, dtype=torch.uint8, device=DEV)
        netcsum.tx_finalize_ip(bt, n, ft, off=o_d, lens=l_d)
        torch.cuda.synchronize()
        _check(bt.cpu().numpy(), tx_w, f"tx bytes ({passes} passes)")
        _check(ft.cpu().numpy(), txf_w, f"tx flags ({passes} passes)")


@pytest.mark.parametrize("form", ["strided", "offlen"])
@pytest.mark.parametrize("bound", [-1, 1, 2])
def test_datagrams_past_the_bitmap_reach(form, bound):
    """Datagrams of 63 000-65 535 B (a run of one may span more than the live-piece bitmap's 63 KiB):
    strided batches take the whole-span form (or the lane-group kernel when a live-piece form is
    forced), offset/length runs the whole-span form for those datagrams; every result the oracle's."""
    netcsum.tune(netcsum.TUNE_PKT_BOUND, bound)
    rng = random.Random(4242 + bound)
    n, slot = 24, 65536 + 128
    pkts = []
    for i in range(n):
        p = make_packet(rng, rng.choice(["tcp", "udp", "icmp", "corrupt_l4"]), payload=rng.randint(62900, 65400))
        pkts.append(p[: 65535])
    buf = np.frombuffer(rng.randbytes(n * slot + 64), np.uint8).copy()
    lead = 5
    for i, p in enumerate(pkts):
        buf[i * slot + lead:i * slot + lead + len(p)] = np.frombuffer(p, np.uint8)
    lens = np.array([len(p) for p in pkts], np.uint16)
    present = 65535
    if form == "strided":
        want = _want(buf, n, slot, lead, present, True)
    else:
        want = _want(buf, n, slot, lead, None, True, lens=lens)
    b = torch.from_numpy(buf).to(DEV)
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    ft = torch.zeros(n, dtype=torch.uint8, device=DEV)
    if form == "strided":
        netcsum.rx_validate_ipv4(b[lead:], n, f, stride=slot, pkt_len=present)
        torch.cuda.synchronize()
        _check(f.cpu().numpy(), want[0], "rx")
        netcsum.tx_finalize_ipv4(b[lead:], n, ft, stride=slot, pkt_len=present)
    else:
        off = torch.from_numpy(np.arange(n, dtype=np.int64) * slot + lead).to(DEV)
        ln = torch.from_numpy(lens.view(np.int16)).to(DEV)
        netcsum.rx_validate_ipv4(b, n, f, off=off, lens=ln)
        torch.cuda.synchronize()
        _check(f.cpu().numpy(), want[0], "rx")
        netcsum.tx_finalize_ipv4(b, n, ft, off=off, lens=ln)
    torch.cuda.synchronize()
    _check(b.cpu().numpy(), want[1], "tx bytes")
    _check(ft.cpu().numpy(), want[2], "tx flags")


def _np_ring(n, slot, lead, sizes, seed, v6_every=0):
    """A ring of n IPv4 TCP / UDP datagrams of the given sizes (numpy-built: the plan needs batches
    of >= 64 Ki frames for its longest runs); every 3rd datagram UDP, headers well-formed, checksum
    fields random (Rx flags then vary), the rest random bytes. v6_every k: every k-th frame IPv6."""
    rng = np.random.default_rng(seed)
    buf = rng.integers(0, 256, size=n * slot + 64, dtype=np.uint8)
    v = buf[: n * slot].reshape(n, slot)
    udp = (np.arange(n) % 3) == 1
    h = v[:, lead:lead + 40]
    h[:, 0], h[:, 1], h[:, 2], h[:, 3] = 0x45, 0, sizes >> 8, sizes & 0xFF
    h[:, 6], h[:, 7], h[:, 8], h[:, 9] = 0x40, 0, 64, np.where(udp, 17, 6)
    h[:, 24] = np.where(udp, (sizes - 20) >> 8, h[:, 24])
    h[:, 25] = np.where(udp, (sizes - 20) & 0xFF, h[:, 25])
    h[:, 32] = np.where(udp, h[:, 32], 0x50)
    if v6_every:
        k = np.arange(n) % v6_every == 0
        pl = sizes - 40
        h[k, 0], h[k, 1], h[k, 2], h[k, 3] = 0x60, 0, 0, 0
        h[k, 4], h[k, 5], h[k, 6], h[k, 7] = (pl[k] >> 8) & 0xFF, pl[k] & 0xFF, 6, 64   # next header TCP
        v[k, lead + 52] = 0x50                                        # its TCP data offset 5 (at +40 + 12)
    return buf


@pytest.mark.parametrize("case", ["template", "ring", "nb2k", "short", "v6mix"])
def test_ring_plan_per_layout_vs_oracle(case):
    """Ring plans (TUNE_PKT_BOUND 4, the default for strided batches of >= 16 Ki frames that are not
    packed): each launch samples 1024 of its datagrams in one extra block (netcsum_pktstream.hip
    pkt_plan_block) and leaves the form and run length for the next batch on the same ring. A ring's
    first batch runs in the host's default (live pieces, runs by slot size); the next ones in the plan:
    full slots the whole-span form 0 (IPv4 runs of 8, mixed-version rings 16), the 40 / 576 / 1500-B
    ring and 300-B frames live pieces in runs of 32, 2-KiB slots live pieces in runs of 8. Every
    batch's Rx flags and Tx bytes equal the oracle's on 2000 sampled frames of a 64 Ki-frame ring (Tx
    in one and two passes), and every frame verifies after the Tx."""
    n = 1 << 16
    rng = np.random.default_rng(7)
    if case == "template":
        slot, lead, sizes, want_plan, v6 = 1520, 14, np.full(n, 1500), "8 bound=0", 0
    elif case == "ring":
        slot, lead, v6 = 1520, 14, 0
        sizes = np.array([40, 576, 1500])[rng.choice(3, size=n, p=[7 / 12, 4 / 12, 1 / 12])]
        want_plan = "32 bound=2"
    elif case == "nb2k":
        slot, lead, sizes, want_plan, v6 = 2048, 64, np.full(n, 1500), "8 bound=2", 0
    elif case == "short":                           # 300-B datagrams in 1520-B slots: 10 KiB / 300 B
        slot, lead, sizes, want_plan, v6 = 1520, 14, np.full(n, 300), "32 bound=2", 0
    else:                                           # IPv4 / IPv6 full frames: RxValidateIP, form 0
        slot, lead, sizes, want_plan, v6 = 1520, 14, np.full(n, 1500), "16 bound=0", 2
    sizes = sizes.astype(np.int64)
    buf = _np_ring(n, slot, lead, sizes, seed=zlib.crc32(case.encode()) & 0xFFFF, v6_every=v6)
    present = slot - lead
    ip = v6 != 0
    rx_fn = netcsum.rx_validate_ip if ip else netcsum.rx_validate_ipv4
    tx_fn = netcsum.tx_finalize_ip if ip else netcsum.tx_finalize_ipv4
    o_rx = op.rx_validate_ip if ip else op.rx_validate
    o_tx = op.tx_finalize_ip if ip else op.tx_finalize
    sample = np.sort(rng.choice(n, size=2000, replace=False))
    want_rx = {int(i): o_rx(bytes(buf[i * slot + lead:i * slot + lead + present])) for i in sample}
    want_tx = {int(i): o_tx(bytes(buf[i * slot + lead:i * slot + lead + present]), True) for i in sample[:600]}
    netcsum.tune(netcsum.TUNE_PKT_BOUND, 4)
    b = torch.from_numpy(buf).to(DEV)
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    launches = []
    for call in range(3):                          # the first batch on the ring, then its plan
        f.zero_()
        rx_fn(b[lead:], n, f, stride=slot, pkt_len=present)
        launches.append(netcsum.last_launch())
        fl = f.cpu().numpy()                       # (synchronises: the plan word is written)
        bad = [i for i, w in want_rx.items() if fl[i] != w]
        assert not bad, (case, call, bad[:5])
    # (the first batch runs in the host's default, or in the plan a previous buffer at the same address
    # left: the plan lags one batch, harmless to the results)
    assert launches[0].endswith("plan=first") or "plan=ring" in launches[0], launches[0]
    for ln in launches[1:]:
        assert "pkts_per_wave=" + want_plan in ln and "plan=ring" in ln, (case, ln)
    ft = torch.zeros(n, dtype=torch.uint8, device=DEV)
    for passes in (1, 2):
        netcsum.tune(netcsum.TUNE_TX_PASSES, passes)
        bt = b.clone()                                            # (a new ring: its first batch,
        tx_fn(bt[lead:], n, ft, stride=slot, pkt_len=present)     # then its plan; Tx is idempotent)
        torch.cuda.synchronize()
        tx_fn(bt[lead:], n, ft, stride=slot, pkt_len=present)
        assert "pkts_per_wave=" + want_plan in netcsum.last_launch(), netcsum.last_launch()
        got = bt.cpu().numpy()
        ftn = ft.cpu().numpy()
        for i, (q, qf) in want_tx.items():
            o = i * slot + lead
            assert bytes(got[o:o + present]) == q and ftn[i] == qf, (case, passes, i)
        f.zero_()
        rx_fn(bt[lead:], n, f, stride=slot, pkt_len=present)
        assert bool(((f & 0x07) == 0x07).all().item()), (case, passes)


@pytest.mark.parametrize("kind", ["rx", "tx1", "tx2"])
def test_deferred_counters_reset_after_a_failed_call(kind):
    """an offset/length batch counts its out-of-order runs in the scratch slot's
    tail words and its deferred pass resets them. A call that fails between the two (here: the
    test-only NETCSUM_TUNE_FAULT_INJECT 1, which enqueues the stream kernel and fails instead of
    launching the deferred pass) leaves them non-zero; the next call on the slot must zero them first,
    or it would re-run the stale list entries (Tx: the same runs twice, concurrently). Shuffled
    descriptors, so every run is listed; the calls after each failure equal the oracle."""
    rng = random.Random(606)
    n, slot, lead = 700, 1520, 14
    buf, lens = _ring(rng, n, slot, lead, v6mix=True)
    perm = np.random.default_rng(9).permutation(n)
    offs = (np.arange(n, dtype=np.int64) * slot + lead)[perm].copy()
    lens = lens[perm].copy()
    o_d = torch.from_numpy(offs).to(DEV)
    l_d = torch.from_numpy(lens.view(np.int16)).to(DEV)
    frames = [bytes(buf[o:o + int(m)]) for o, m in zip(offs.tolist(), lens.tolist())]
    if kind == "rx":
        want = np.array([op.rx_validate_ip(f) for f in frames], np.uint8)
    else:
        netcsum.tune(netcsum.TUNE_TX_PASSES, 1 if kind == "tx1" else 2)
        want = buf.copy()
        want_f = np.zeros(n, np.uint8)
        for i, (o, m) in enumerate(zip(offs.tolist(), lens.tolist())):
            q, want_f[i] = op.tx_finalize_ip(bytes(buf[o:o + int(m)]), True)
            want[o:o + int(m)] = np.frombuffer(q, np.uint8)

    def call(check=True):
        f = torch.zeros(n, dtype=torch.uint8, device=DEV)
        if kind == "rx":
            err = netcsum.rx_validate_ip(torch.from_numpy(buf).to(DEV), n, f, off=o_d, lens=l_d, check=check)
            torch.cuda.synchronize()
            return err, f.cpu().numpy(), None
        bt = torch.from_numpy(buf).to(DEV)
        err = netcsum.tx_finalize_ip(bt, n, f, off=o_d, lens=l_d, check=check)
        torch.cuda.synchronize()
        return err, bt.cpu().numpy(), f.cpu().numpy()

    try:
        for rep in range(3):
            netcsum.tune(netcsum.TUNE_FAULT_INJECT, 1)
            err, _, _ = call(check=False)
            assert err == netcsum.NET_UTIL_ERR_MI355X_DEV, err
            assert "offlen +pkt_vl_deferred_kernel" in netcsum.last_launch(), netcsum.last_launch()
            for _ in range(2):
                err, got, got_f = call()
                assert err == netcsum.NET_UTIL_ERR_NONE, err
                _check(got, want, f"{kind} after failed call {rep}")
                if got_f is not None:
                    _check(got_f, want_f, f"{kind} flags after failed call {rep}")
    finally:
        netcsum.tune(netcsum.TUNE_FAULT_INJECT, 0)
