"""GPU parity of the IPv4 packet batches (fused Rx validation, Tx finalize with write-back) against
the packet oracle, which composes the C oracle's reference functions per packet."""
import random

import numpy as np
import pytest

import netcsum
import oracle_packets as op
from packets import KINDS, make_packet, packed_batch

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _defaults():
    for k in (netcsum.TUNE_GRID_BLOCKS, netcsum.TUNE_GROUP_LANES):
        netcsum.tune(k, 0)
    netcsum.tune(netcsum.TUNE_NT_LOADS, -1)
    netcsum.tune(netcsum.TUNE_TILE, -1)
    yield
    for k in (netcsum.TUNE_GRID_BLOCKS, netcsum.TUNE_GROUP_LANES):
        netcsum.tune(k, 0)
    netcsum.tune(netcsum.TUNE_NT_LOADS, -1)
    netcsum.tune(netcsum.TUNE_TILE, -1)


def _rx_gpu(buf, offs, lens):
    b = torch.from_numpy(buf).to(DEV)
    o = torch.from_numpy(offs.view(np.int64)).to(DEV)
    ln = torch.from_numpy(lens.view(np.int16)).to(DEV)
    f = torch.zeros(len(offs), dtype=torch.uint8, device=DEV)
    netcsum.rx_validate_ipv4(b, len(offs), f, off=o, lens=ln)
    torch.cuda.synchronize()
    return f.cpu().numpy()


@pytest.mark.parametrize("group", [0, 8, 16, 32, 64])
@pytest.mark.parametrize("grid,tile", [(0, -1), (3, 0)])
def test_rx_validate_mixed_varlen(group, grid, tile):
    rng = random.Random(group * 7 + grid)
    pkts = [make_packet(rng, rng.choice(KINDS)) for _ in range(1500)]
    buf, offs, lens = packed_batch(pkts, rng)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
    netcsum.tune(netcsum.TUNE_TILE, tile)
    got = _rx_gpu(buf, offs, lens)
    want = np.array([op.rx_validate(bytes(buf[o:o + n])) for o, n in zip(offs.tolist(), lens.tolist())], np.uint8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(pkts[i][:24].hex(), int(got[i]), int(want[i])) for i in bad[:5]]


def test_rx_validate_strided_c2_shape():
    """1500-B TCP datagrams in a strided batch (the C2 shape with real IP/TCP headers)."""
    rng = random.Random(11)
    n = 4000
    pkts = [make_packet(rng, rng.choice(["tcp", "tcp", "corrupt_l4", "corrupt_ip"]), payload=1500 - 40)
            for _ in range(n)]
    L = 1500
    buf = np.zeros(n * L + 64, np.uint8)
    for i, p in enumerate(pkts):
        p = p[:L]
        buf[i * L:i * L + len(p)] = np.frombuffer(p, np.uint8)
    b = torch.from_numpy(buf).to(DEV)
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.rx_validate_ipv4(b, n, f, stride=L, pkt_len=L)
    torch.cuda.synchronize()
    want = np.array([op.rx_validate(bytes(buf[i * L:(i + 1) * L])) for i in range(n)], np.uint8)
    assert np.array_equal(f.cpu().numpy(), want)


@pytest.mark.parametrize("udp_tx_csum", [True, False])
def test_tx_finalize_writes_reference_checksums_then_rx_accepts(udp_tx_csum):
    rng = random.Random(21 + udp_tx_csum)
    kinds = ["tcp", "udp", "udp", "icmp", "igmp", "other", "frag", "udp_badlen", "tcp_short", "bad_ver"]
    pkts = []
    for _ in range(2000):
        p = bytearray(make_packet(rng, rng.choice(kinds)))
        if len(p) >= 12 and rng.random() < 0.5:
            p[10:12] = bytes([rng.getrandbits(8), rng.getrandbits(8)])   # stale checksum fields
        pkts.append(bytes(p))
    buf, offs, lens = packed_batch(pkts, rng)
    b = torch.from_numpy(buf).to(DEV)
    o = torch.from_numpy(offs.view(np.int64)).to(DEV)
    ln = torch.from_numpy(lens.view(np.int16)).to(DEV)
    f = torch.zeros(len(pkts), dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv4(b, len(pkts), f, off=o, lens=ln, udp_tx_csum=udp_tx_csum)
    torch.cuda.synchronize()
    out = b.cpu().numpy()
    flags = f.cpu().numpy()
    for i, (off, n) in enumerate(zip(offs.tolist(), lens.tolist())):
        pkt = bytes(buf[off:off + n])
        want_pkt, want_f = op.tx_finalize(pkt, udp_tx_csum)
        assert bytes(out[off:off + n]) == want_pkt, (i, pkt[:24].hex())
        assert flags[i] == want_f, (i, flags[i], want_f)
    # the finalized batch validates on the GPU Rx path
    got = _rx_gpu(out, offs, lens)
    ok = ((got & op.MALFORMED) == 0)
    assert ((got[ok] & op.IP_OK) != 0).all()
    checked = ok & ((got & op.L4_CHECKED) != 0)
    assert ((got[checked] & op.L4_OK) != 0).all()


@pytest.mark.parametrize("stride,pkt_len", [(1500, 1500), (1540, 1514), (2048, 1514), (200, 184), (192, 48)])
@pytest.mark.parametrize("group", [0, 16, 32])
def test_tx_finalize_strided_vs_oracle(stride, pkt_len, group):
    """Strided Tx finalize (uniform buffer stores addressed from the wave's first packet): packets
    finalized exactly as the packet oracle does, and every byte between packets (stride > pkt_len)
    and past the last one left as it was; strides that are not multiples of 16 put packets at every
    alignment; lane groups of 16 / 32 (and the auto choice, 8 lanes for small packets)."""
    rng = random.Random(stride * 7 + pkt_len * 3 + group)
    n = 600
    kinds = ["tcp", "tcp", "udp", "udp0", "icmp", "igmp", "other", "frag", "tcp_short", "bad_ver"]
    buf = np.frombuffer(rng.randbytes(n * stride + 64), np.uint8).copy()
    for i in range(n):
        p = bytearray(make_packet(rng, rng.choice(kinds), payload=rng.randint(0, max(0, pkt_len - 100))))
        p = p[:pkt_len]
        if len(p) >= 12 and rng.random() < 0.5:
            p[10:12] = rng.randbytes(2)                           # stale IP checksum field
        buf[i * stride:i * stride + len(p)] = np.frombuffer(bytes(p), np.uint8)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    b = torch.from_numpy(buf).to(DEV)
    assert b.data_ptr() % 64 == 0
    f = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv4(b, n, f, stride=stride, pkt_len=pkt_len)
    torch.cuda.synchronize()
    out = b.cpu().numpy()
    want = buf.copy()
    want_f = np.zeros(n, np.uint8)
    for i in range(n):
        pk, want_f[i] = op.tx_finalize(bytes(buf[i * stride:i * stride + pkt_len]), True)
        want[i * stride:i * stride + pkt_len] = np.frombuffer(pk, np.uint8)
    bad = np.nonzero(out != want)[0]
    assert bad.size == 0, [(int(j), int(j) // stride, int(j) % stride, int(out[j]), int(want[j])) for j in bad[:8]]
    assert np.array_equal(f.cpu().numpy(), want_f)


@pytest.mark.parametrize("group", [0, 64])
def test_ipv4_extreme_sizes(group):
    """IPv4 datagrams at the size limits: 20-B header only, minimal UDP / TCP / ICMP, and total
    lengths up to 65535 B (the 16-bit limit) with and without IP options, packed at odd offsets;
    Rx verdicts and Tx write-back equal the packet oracle."""
    rng = random.Random(950 + group)
    pkts = [make_packet(rng, "other", payload=0), make_packet(rng, "udp", payload=0),
            make_packet(rng, "tcp", payload=0), make_packet(rng, "icmp", payload=0)]
    for kind in ("tcp", "udp", "icmp", "tcp"):
        p = make_packet(rng, kind, payload=0)
        room = 65535 - len(p)
        pkts.append(make_packet(random.Random(rng.random()), kind, payload=0))
        big = None
        for _ in range(20):                                      # options / TCP header length vary
            r = random.Random(rng.random())
            cand = make_packet(r, kind, payload=room - 60)
            if len(cand) <= 65535:
                big = cand
                break
        assert big is not None
        pkts.append(big)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    buf, offs, lens = packed_batch(pkts, rng, trailer=False)
    got = _rx_gpu(buf, offs, lens)
    want = np.array([op.rx_validate(bytes(buf[o:o + n])) for o, n in zip(offs.tolist(), lens.tolist())], np.uint8)
    assert np.array_equal(got, want), (got, want)
    b = torch.from_numpy(buf).to(DEV)
    o_ = torch.from_numpy(offs.view(np.int64)).to(DEV)
    ln = torch.from_numpy(lens.view(np.int16)).to(DEV)
    f = torch.zeros(len(pkts), dtype=torch.uint8, device=DEV)
    netcsum.tx_finalize_ipv4(b, len(pkts), f, off=o_, lens=ln)
    torch.cuda.synchronize()
    out = b.cpu().numpy()
    for i, (o, n) in enumerate(zip(offs.tolist(), lens.tolist())):
        want_pkt, want_f = op.tx_finalize(bytes(buf[o:o + n]), True)
        assert bytes(out[o:o + n]) == want_pkt, i
        assert f.cpu().numpy()[i] == want_f, i
