"""Every single-GPU BASELINE config at FULL size on the GPU (the 8-GPU C5 run itself is the driver's):

* C5 per-GPU shard — 16 M x 1500-B TCP segments + 12-B pseudo-headers (25.4 GB resident);
* C3 — 16 M x 20-B IPv4 headers, HdrCalc / HdrVerify;
* C4 — 1 M packed UDP datagrams of U{40..9000} B (PRNG seed 7, odd starts) + 12-B pseudo-headers.

Each runs the size-independent properties the domain offers — Calc, write the value into the
checksum field the reference's callers write (NET_UTIL_VAL_COPY_16: net_tcp.c:29862 at TCP offset 16,
net_ipv4.c:9586 at IPv4 offset 10, net_udp.c:2937 at UDP offset 6), then Verify EVERY element OK;
one corrupted byte in every 1000th element is detected exactly — plus a bit-exact oracle comparison
of 4096 sampled elements (oracle = the C restatement of net_util.c, test infrastructure only).
"""
import numpy as np
import pytest

import netcsum
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"
SEED = 0x5EED0001


def _out(n, op):
    return torch.zeros(n, dtype=torch.int16 if op in (0, 2) else torch.uint8, device=DEV)


def _np16(t):
    return t.cpu().numpy().view(np.uint16)


def _sample(n, k=4096, seed=1):
    return np.sort(np.random.default_rng(seed).choice(n, size=k, replace=False))


def _pseudo(n, L, proto):
    idx = torch.arange(n, device=DEV, dtype=torch.int64)
    ph = torch.zeros(n, 12, dtype=torch.uint8, device=DEV)
    for b in range(4):
        ph[:, b] = ((idx >> (8 * (3 - b))) & 0xFF).to(torch.uint8)
        ph[:, 4 + b] = (((idx * 2654435761) >> (8 * (3 - b))) & 0xFF).to(torch.uint8)
    ph[:, 9] = proto
    if isinstance(L, int):
        ph[:, 10], ph[:, 11] = L >> 8, L & 0xFF
    else:
        ph[:, 10], ph[:, 11] = (L >> 8).to(torch.uint8), (L & 0xFF).to(torch.uint8)
    return ph.reshape(-1).contiguous()


def _check_corruption(run_verify, corrupt, n):
    bad = torch.arange(0, n, 1000, device=DEV)
    corrupt(bad)
    ok = run_verify()
    failed = torch.nonzero(ok == 0).flatten()
    assert torch.equal(failed, bad), (failed[:8].tolist(), bad[:8].tolist())


def test_c5_shard_16M_x_1500B():
    n, L = 1 << 24, 1500
    seg = torch.empty(n * L + 256, dtype=torch.uint8, device=DEV)
    netcsum.fill(seg, n * L, SEED, 0)
    ph = _pseudo(n, L, 6)
    s2 = seg[: n * L].view(n, L)
    csum = _out(n, 0)
    netcsum.batch_strided(seg, L, L, ph, 12, 12, n, csum, 0)
    torch.cuda.synchronize()
    smp = _sample(n)
    sidx = torch.from_numpy(smp).to(DEV)
    want = oracle.batch_strided(s2[sidx].cpu().numpy().reshape(-1), L, L, ph.view(n, 12)[sidx].cpu().numpy().reshape(-1),
                                12, 12, len(smp), 0)
    assert np.array_equal(_np16(csum)[smp], want)
    # Tx -> Rx: zero the TCP checksum field, Calc, store (host-order value, memcpy), Verify all
    s2[:, 16:18] = 0
    netcsum.batch_strided(seg, L, L, ph, 12, 12, n, csum, 0)
    s2[:, 16:18] = csum.view(torch.uint8).view(n, 2)
    ok = _out(n, 1)

    def verify():
        netcsum.batch_strided(seg, L, L, ph, 12, 12, n, ok, 1)
        torch.cuda.synchronize()
        return ok

    assert bool(verify().all())

    def corrupt(bad):
        s2[bad, 1001] ^= 0x01

    _check_corruption(verify, corrupt, n)


def test_c3_16M_x_20B_headers():
    n, L = 1 << 24, 20
    hdr = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    netcsum.fill(hdr, n * L, SEED + 3, 0)
    h2 = hdr.view(n, L)
    h2[:, 0] = 0x45
    csum = _out(n, 2)
    netcsum.batch_strided(hdr, L, L, None, 0, 0, n, csum, 2)
    torch.cuda.synchronize()
    smp = _sample(n)
    host = h2[torch.from_numpy(smp).to(DEV)].cpu().numpy().reshape(-1)
    for op in (2, 3):
        got = _out(n, op)
        netcsum.batch_strided(hdr, L, L, None, 0, 0, n, got, op)
        torch.cuda.synchronize()
        want = oracle.batch_strided(host, L, L, None, 0, 0, len(smp), op)
        g = got.cpu().numpy()
        assert np.array_equal(g.view(np.uint16)[smp] if op == 2 else g[smp], want), op
    # IPv4 Tx -> Rx (net_ipv4.c:9573-9586 then :5247): zero the field, HdrCalc, store, HdrVerify all
    h2[:, 10:12] = 0
    netcsum.batch_strided(hdr, L, L, None, 0, 0, n, csum, 2)
    h2[:, 10:12] = csum.view(torch.uint8).view(n, 2)
    ok = _out(n, 3)

    def verify():
        netcsum.batch_strided(hdr, L, L, None, 0, 0, n, ok, 3)
        torch.cuda.synchronize()
        return ok

    assert bool(verify().all())

    def corrupt(bad):
        h2[bad, 8] ^= 0x80                               # TTL

    _check_corruption(verify, corrupt, n)


def test_c4_1M_packed_udp_40_9000B():
    n = 1 << 20
    rng = np.random.default_rng(7)
    lens = rng.integers(40, 9001, size=n).astype(np.uint16)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    total = int(off[-1]) + int(lens[-1])
    assert (off & 1).sum() > n // 3                            # packed: ~half the starts are odd
    base = torch.empty(total + 256, dtype=torch.uint8, device=DEV)
    netcsum.fill(base, total, SEED + 4, 0)
    off_d = torch.from_numpy(off.view(np.int64)).to(DEV)
    len_d = torch.from_numpy(lens.view(np.int16)).to(DEV)
    len64 = torch.from_numpy(lens.astype(np.int64)).to(DEV)
    ph = _pseudo(n, len64, 17)
    csum = _out(n, 0)
    netcsum.batch_varlen(base, off_d, len_d, ph, 12, 12, n, csum, 0)
    torch.cuda.synchronize()
    # sampled oracle comparison: gather the sampled datagrams into one host buffer
    smp = _sample(n)
    s_off, s_len = off[smp].astype(np.int64), lens[smp].astype(np.int64)
    s_len_d = torch.from_numpy(s_len).to(DEV)
    starts = torch.repeat_interleave(torch.from_numpy(s_off).to(DEV), s_len_d)
    first = torch.repeat_interleave(torch.cumsum(s_len_d, 0) - s_len_d, s_len_d)
    pos = starts + torch.arange(int(s_len.sum()), device=DEV) - first
    host = base[pos].cpu().numpy()
    h_off = np.zeros(len(smp), np.uint64)
    h_off[1:] = np.cumsum(s_len[:-1]).astype(np.uint64)
    want = oracle.batch_varlen(host, h_off, s_len.astype(np.uint16),
                               ph.view(n, 12)[torch.from_numpy(smp).to(DEV)].cpu().numpy().reshape(-1), 12, 12, 0)
    assert np.array_equal(_np16(csum)[smp], want)
    # UDP Tx -> Rx: zero the checksum field (datagram bytes 6-7), DataCalc, store, DataVerify all
    f0 = off_d + 6
    base[f0] = 0
    base[f0 + 1] = 0
    netcsum.batch_varlen(base, off_d, len_d, ph, 12, 12, n, csum, 0)
    cb = csum.view(torch.uint8).view(n, 2)
    base[f0] = cb[:, 0]
    base[f0 + 1] = cb[:, 1]
    ok = _out(n, 1)

    def verify():
        netcsum.batch_varlen(base, off_d, len_d, ph, 12, 12, n, ok, 1)
        torch.cuda.synchronize()
        return ok

    assert bool(verify().all())

    def corrupt(bad):
        p = off_d[bad] + (len64[bad] // 2)
        base[p] ^= 0x10

    _check_corruption(verify, corrupt, n)
