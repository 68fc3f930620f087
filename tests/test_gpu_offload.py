"""GPU parity of the checksum-offload burst adapters (include/netcsum_mi355x.h (2b'')):

* NetUtil_MI355X_RxBurst on mixed IPv4 / IPv6 bursts — strided (the run-stream kernel) and packed
  offset/length (the lane-group kernel), IPv6 chains past every window (the walk pass), with and
  without a flags array, with and without NET_UDP_CFG_RX_CHK_SUM_DISCARD_EN: each frame's action
  equals NetUtil_MI355X_RxAction of the oracle's verdict (oracle/oracle_packets.py), its flags the
  oracle's, and its decision the reference's (oracle/oracle_offload.py rx_reference, offload flags
  off) once the stack built with the offload flags has seen the delivered frames.
* NetUtil_MI355X_TxBurst on the frames the stack builds with the Tx offload flags (0 in the IPv4 /
  TCP / ICMPv4 fields, the UDP placeholder 0xFFFF, 0 for "no UDP checksum") rebuilds, in place, the
  frames the reference builds with the flags off; nothing outside the fields changes.
"""
import random

import numpy as np
import pytest

import netcsum
import oracle_offload as oo
import oracle_packets as op
from packets import KINDS, KINDS6, make_packet, make_packet_v6, packed_batch

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"


def _mixed(rng, n, max_payload, long_chains=True):
    out = []
    for i in range(n):
        if rng.random() < 0.5:
            out.append(make_packet(rng, rng.choice(KINDS), payload=rng.randint(0, max_payload)))
        else:
            kinds = KINDS6 if long_chains else [k for k in KINDS6 if k != "ext_long"]
            out.append(make_packet_v6(rng, rng.choice(kinds), payload=rng.randint(0, max_payload)))
    for mk in (make_packet, make_packet_v6):                     # corrupted UDP, both versions
        for _ in range(max(1, n // 40)):
            u = bytearray(mk(rng, "udp", payload=rng.randint(1, max_payload)))
            u[-1] ^= 1 << rng.randint(0, 7)
            out.append(bytes(u))
    rng.shuffle(out)
    return out


def _want_actions(pkts, cfg):
    f = np.array([op.rx_validate_ip(p) for p in pkts], np.uint8)
    a = np.array([netcsum.rx_action(int(x), oo.transport_proto(p), len(p) and p[0] >> 4 == 6, cfg)
                  for x, p in zip(f, pkts)], np.uint8)
    return f, a


def _check_decisions(pkts, acts, discard):
    for k, (p, a) in enumerate(zip(pkts, acts)):
        want = oo.rx_reference(p, udp_discard=discard)
        got = oo.rx_with_adapter(p, int(a), udp_discard=discard)
        assert got[0] == want[0], (k, want, got, int(a))
        if want[0] == "drop" and want[1] in oo.CHECKSUM_COUNTERS:
            assert got[1] == want[1], (k, want, got)


@pytest.mark.parametrize("discard", [False, True])
@pytest.mark.parametrize("with_flags", [True, False])
def test_rx_burst_varlen(discard, with_flags):
    rng = random.Random(10 + discard + 2 * with_flags)
    pkts = _mixed(rng, 900, 1400)
    cfg = netcsum.RXCFG_UDP_DISCARD_NO_CHK_SUM if discard else 0
    buf, offs, lens = packed_batch(pkts, rng)
    b = torch.from_numpy(buf).to(DEV)
    o = torch.from_numpy(offs.astype(np.int64)).to(DEV)
    ln = torch.from_numpy(lens.view(np.int16)).to(DEV)
    n = len(pkts)
    act = torch.full((n,), 0xEE, dtype=torch.uint8, device=DEV)
    fl = torch.zeros(n, dtype=torch.uint8, device=DEV) if with_flags else None
    netcsum.rx_burst(b, n, act, flags=fl, off=o, lens=ln, rx_cfg=cfg)
    torch.cuda.synchronize()
    want_f, want_a = _want_actions([bytes(buf[x:x + y]) for x, y in zip(offs, lens)], cfg)
    got_a = act.cpu().numpy()
    assert np.array_equal(got_a, want_a), np.nonzero(got_a != want_a)[0][:10]
    if with_flags:
        assert np.array_equal(fl.cpu().numpy(), want_f)
    _check_decisions([bytes(buf[x:x + y]) for x, y in zip(offs, lens)], got_a, discard)
    counts = netcsum.rx_burst_tally(got_a)
    assert sum(counts) == n and counts[netcsum.RX_DROP_TCP_CHK_SUM] > 0 and counts[netcsum.RX_DROP_UDP_CHK_SUM] > 0


@pytest.mark.parametrize("stride,pkt_len,lead", [(1500, 1500, 0), (1536, 1500, 1), (576, 576, 3), (2048, 1514, 2)])
def test_rx_burst_strided(stride, pkt_len, lead):
    rng = random.Random(stride + lead)
    n = 700
    pkts = _mixed(rng, n, pkt_len - 100)[:n]
    buf = np.frombuffer(rng.randbytes(lead + n * stride + 96), np.uint8).copy()
    for i, p in enumerate(pkts):
        p = p[:pkt_len]
        buf[lead + i * stride:lead + i * stride + len(p)] = np.frombuffer(p, np.uint8)
    b = torch.from_numpy(buf).to(DEV)
    act = torch.full((n,), 0xEE, dtype=torch.uint8, device=DEV)
    fl = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.rx_burst(b[lead:], n, act, flags=fl, stride=stride, pkt_len=pkt_len)
    torch.cuda.synchronize()
    frames = [bytes(buf[lead + i * stride:lead + i * stride + pkt_len]) for i in range(n)]
    want_f, want_a = _want_actions(frames, 0)
    assert np.array_equal(fl.cpu().numpy(), want_f)
    assert np.array_equal(act.cpu().numpy(), want_a)
    _check_decisions(frames, act.cpu().numpy(), False)


def test_rx_burst_lane_group_kernel_and_errors():
    rng = random.Random(5)
    n = 300
    pkts = _mixed(rng, n, 1300)[:n]
    stride = 1500
    buf = np.zeros(n * stride + 64, np.uint8)
    for i, p in enumerate(pkts):
        buf[i * stride:i * stride + len(p[:stride])] = np.frombuffer(p[:stride], np.uint8)
    b = torch.from_numpy(buf).to(DEV)
    act = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tune(netcsum.TUNE_KERNEL, 2)
    try:
        netcsum.rx_burst(b, n, act, stride=stride, pkt_len=stride)
        torch.cuda.synchronize()
    finally:
        netcsum.tune(netcsum.TUNE_KERNEL, 0)
    _, want_a = _want_actions([bytes(buf[i * stride:(i + 1) * stride]) for i in range(n)], 0)
    assert np.array_equal(act.cpu().numpy(), want_a)
    L = netcsum.lib()
    assert L.NetUtil_MI355X_RxBurst(b.data_ptr(), None, None, stride, stride, n, 0, None, None, None) == \
        netcsum.NET_ERR_FAULT_NULL_PTR
    assert L.NetUtil_MI355X_RxBurst(b.data_ptr(), None, None, stride, stride, n, 2, act.data_ptr(), None, None) == \
        netcsum.NET_UTIL_ERR_MI355X_INVALID_ARG


def _tx_frames(rng, n, max_payload):
    out = []
    for i in range(n):
        csum = rng.random() < 0.8                                 # per datagram: NET_UDP_FLAG_TX_CHK_SUM_DIS
        if i % 2:
            kind = rng.choice(["tcp", "udp", "udp", "icmp", "igmp", "other", "frag"])
            pkt = make_packet(rng, kind, payload=rng.randint(0, max_payload))
        else:
            kind = rng.choice(["tcp", "udp", "udp", "icmp_echo", "icmp_err", "icmp_nd", "other", "ext_ok",
                               "ext_frag", "ext_long"])
            pkt = make_packet_v6(rng, kind, payload=rng.randint(0, max_payload))
        out.append((oo.tx_stack_offload(pkt, csum), op.tx_finalize_ip(pkt, csum)[0]))
    return out


def test_tx_burst_varlen_rebuilds_reference_frames():
    rng = random.Random(21)
    pairs = _tx_frames(rng, 800, 1400)
    buf, offs, lens = packed_batch([f for f, _ in pairs], rng, trailer=False)
    want = buf.copy()
    for (_, r), x in zip(pairs, offs):
        want[x:x + len(r)] = np.frombuffer(r, np.uint8)
    b = torch.from_numpy(buf).to(DEV)
    netcsum.tx_burst(b, len(pairs), off=torch.from_numpy(offs.astype(np.int64)).to(DEV),
                     lens=torch.from_numpy(lens.view(np.int16)).to(DEV))
    torch.cuda.synchronize()
    got = b.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:16]


@pytest.mark.parametrize("stride,pkt_len,two_pass", [(1500, 1500, True), (1500, 1500, False), (2048, 1514, True),
                                                     (640, 600, True)])
def test_tx_burst_strided_rebuilds_reference_frames(stride, pkt_len, two_pass):
    rng = random.Random(stride + pkt_len)
    n = 600
    pairs = _tx_frames(rng, n, pkt_len - 120)
    buf = np.frombuffer(rng.randbytes(n * stride + 64), np.uint8).copy()
    for i, (f, _) in enumerate(pairs):
        f = f[:pkt_len]
        buf[i * stride:i * stride + len(f)] = np.frombuffer(f, np.uint8)
    # the slot's bytes as the adapter's rule finalizes them: the reference frame where it fits (a
    # frame cut by the slot is finalized as its truncated bytes dictate)
    want = buf.copy()
    for i, (f, r) in enumerate(pairs):
        slot = bytes(buf[i * stride:i * stride + pkt_len])
        fin = oo.tx_burst_model(slot)
        if len(f) <= pkt_len:
            assert fin[:len(r)] == r, i
        want[i * stride:i * stride + pkt_len] = np.frombuffer(fin, np.uint8)
    b = torch.from_numpy(buf).to(DEV)
    fl = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tune(netcsum.TUNE_TX_PASSES, 2 if two_pass else 1)
    try:
        netcsum.tx_burst(b, n, flags=fl, stride=stride, pkt_len=pkt_len)
        torch.cuda.synchronize()
    finally:
        netcsum.tune(netcsum.TUNE_TX_PASSES, 0)
    got = b.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:16]
