"""GPU parity of the CRC-32 path (net_util.c:485-636): the drop-in NetUtil_32BitCRC_Calc / _CalcCpl
on host buffers (GPU past 4096 octets), the drivers' multicast hash built on them, and the strided / varlen batch kernels
(one lane per short segment; for long ones 16-lane groups over interleaved 16-B chunks with table-driven
shifts, the default, or over equal blocks combined by GF(2) multiplications, NETCSUM_TUNE_CRC_KERNEL 1),
against the C restatement (pinned to the CRC-32 check value and zlib in tests/test_crc_cpu.py).
Full size: the Ethernet residue property — a segment followed by its little-endian CalcCpl value
has CalcCpl 0x2144DF1C — over every segment of a 1 M x 1500-B batch."""
import ctypes
import random

import numpy as np
import pytest

import netcsum
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"
RESIDUE = int(np.array([0x2144DF1C], np.uint32).view(np.int32)[0])   # CRC-32 residue, as the int32 out holds it


def _host(data: bytes):
    buf = (ctypes.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    return buf, ctypes.addressof(buf)


@pytest.mark.parametrize("cpl", [False, True])
def test_dropin_crc_vs_oracle(cpl):
    """Calls of up to 4096 octets run the reference's register update on the host (the per-call MAC
    hash), longer ones go through the GPU kernel (NetUtil_MI355X_CRC32Host): both equal the oracle."""
    rng = random.Random(11 + cpl)
    for n in list(range(1, 80)) + [255, 256, 257, 1023, 1500, 4095, 4096, 4097, 9000, 65535, 65536, 200003]:
        m = rng.randbytes(n)
        keep, p = _host(m)
        for off in [o for o in ((0, 1, 3) if n < 300 else (0, 5)) if o < n]:
            got = netcsum.CRC32Calc(p + off, n - off, cpl)
            want = oracle.crc32_calc(m[off:], cpl)
            assert got == want, (n, off, hex(got[0]), hex(want[0]))
    keep, p = _host(b"123456789")                                  # keep the buffer alive
    assert netcsum.CRC32Calc(p, 9, True) == (0xCBF43926, netcsum.NET_UTIL_ERR_NONE)


def test_dropin_multicast_hash_like_the_drivers():
    """Dev/Ether/GMAC/net_dev_gmac.c:2673-2683: hash = Reflect(CalcCpl(mac, 6)) >> 26."""
    rng = random.Random(3)
    for _ in range(64):
        mac = bytes([0x01, 0x00, 0x5E]) + rng.randbytes(3)
        keep, p = _host(mac)
        crc, err = netcsum.CRC32Calc(p, 6, True)
        assert err == netcsum.NET_UTIL_ERR_NONE
        want, _ = oracle.crc32_calc(mac, True)
        assert (netcsum.Reflect32(crc) >> 26) & 0x3F == (oracle.reflect32(want) >> 26) & 0x3F


# (NETCSUM_TUNE_CRC_KERNEL, _NT, _LANES, _WIDE): auto, block combine, interleaved for every length (nt),
# one lane per segment for every length, interleaved with 1 .. 16 lanes per segment; byte (0), 11-bit (1) or
# lane-replicated 6-bit (2) tables
# The matrix guards the shipped forms (auto: tiny / lane / interleaved with 11-bit tables) and one
# variant per alternative kernel a TUNE key selects; round 2's sweeps of every lane count and table
# form are recorded in DESIGN.md and not re-run here.
FORMS = [(0, 0, 0, 1), (1, 0, 0, 1), (2, 1, 0, 1), (3, 0, 0, 1), (2, 0, 16, 0), (2, 0, 1, 2)]


def expected_kernel(form, length, varlen=False):
    kern, nt, lanes, wide = form
    short = length <= 96 and not varlen
    if kern == 3 or (kern in (0, 1) and short):
        return "crc_tiny_kernel " if (length <= 16 and not varlen) else "crc_lane_kernel "
    if kern == 1:
        return "crc_group_kernel G=16 "
    tag = ",".join(t for t, on in (("nt", nt), ("w11", wide == 1), ("k6", wide == 2)) if on)
    auto = 8 if (length >= 1024 and not varlen) else 4
    return "crc_ilv_kernel" + (f"<{tag}>" if tag else "") + f" G={lanes or auto} "


@pytest.fixture(params=FORMS, ids=lambda f: "k{}nt{}g{}w{}".format(*f))
def crc_form(request):
    kern, nt, lanes, wide = request.param
    netcsum.tune(netcsum.TUNE_CRC_KERNEL, kern)
    netcsum.tune(netcsum.TUNE_CRC_NT, nt)
    netcsum.tune(netcsum.TUNE_CRC_LANES, lanes)
    netcsum.tune(netcsum.TUNE_CRC_WIDE, wide)
    yield request.param
    netcsum.tune(netcsum.TUNE_CRC_KERNEL, 0)
    netcsum.tune(netcsum.TUNE_CRC_NT, 0)
    netcsum.tune(netcsum.TUNE_CRC_LANES, 0)
    netcsum.tune(netcsum.TUNE_CRC_WIDE, 1)


STRIDED = [(6, 6), (6, 8), (1, 1), (16, 16), (17, 20), (96, 96), (97, 100), (257, 300), (1500, 1500), (1514, 1518),
           (9000, 9001), (65535, 65536)]


@pytest.mark.parametrize("length,stride", STRIDED)
@pytest.mark.parametrize("cpl", [0, 1])
def test_crc_batch_strided_vs_oracle(length, stride, cpl, crc_form):
    rng = np.random.default_rng(length * 3 + stride + cpl)
    n = 1000 if length <= 1514 else 200 if length <= 9001 else 24
    for base_off in (0, 1, 13):
        data = rng.integers(0, 256, size=base_off + n * stride + 64, dtype=np.uint8)
        d = torch.from_numpy(data).to(DEV)
        out = torch.zeros(n, dtype=torch.int32, device=DEV)
        netcsum.crc32_strided(d.data_ptr() + base_off, stride, length, n, out, cpl)
        torch.cuda.synchronize()
        want = oracle.crc32_batch(data[base_off:].copy(), n, bool(cpl), stride=stride, length=length)
        got = out.cpu().numpy().view(np.uint32)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (base_off, [(int(i), hex(got[i]), hex(want[i])) for i in bad[:4]])
        kern = netcsum.last_launch()
        assert kern.startswith(expected_kernel(crc_form, length)), kern


@pytest.mark.parametrize("cpl", [0, 1])
def test_crc_batch_varlen_vs_oracle(cpl, crc_form):
    """Packed segments of 0..20000 B at every alignment, reversed and overlapping layouts."""
    rng = np.random.default_rng(40 + cpl)
    n = 3000
    lens = rng.integers(0, 3000, size=n).astype(np.uint32)
    lens[::97] = rng.integers(9000, 20000, size=len(lens[::97]))
    lens[::53] = 0
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    off += 3
    for layout in ("packed", "reversed", "overlap"):
        o, ln = off.copy(), lens.copy()
        if layout == "reversed":
            o, ln = o[::-1].copy(), ln[::-1].copy()
        elif layout == "overlap":
            o = (o // 3).astype(np.uint64)
        tot = int((o + ln).max()) + 64
        data = rng.integers(0, 256, size=tot, dtype=np.uint8)
        d = torch.from_numpy(data).to(DEV)
        od = torch.from_numpy(o.view(np.int64)).to(DEV)
        ld = torch.from_numpy(ln.view(np.int32)).to(DEV)
        out = torch.zeros(n, dtype=torch.int32, device=DEV)
        netcsum.crc32_varlen(d, od, ld, n, out, cpl)
        torch.cuda.synchronize()
        want = oracle.crc32_batch(data, n, bool(cpl), off=o, lens=ln)
        got = out.cpu().numpy().view(np.uint32)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (layout, [(int(i), int(ln[i]), hex(got[i]), hex(want[i])) for i in bad[:4]])


def test_crc_full_size_residue_1M():
    """1 M x 1500-B frames (stride 1504): CalcCpl of each, written little-endian after it, then
    CalcCpl over the 1504 bytes is the CRC-32 residue 0x2144DF1C for every frame; one flipped bit per
    1000 frames breaks exactly those; 4096 sampled frames equal the oracle."""
    n, L, S = 1 << 20, 1500, 1504
    buf = torch.empty(n * S + 64, dtype=torch.uint8, device=DEV)
    netcsum.fill(buf, n * S, 0x5EED00C3, 0)
    fcs = torch.zeros(n, dtype=torch.int32, device=DEV)
    netcsum.crc32_strided(buf, S, L, n, fcs, 1)
    torch.cuda.synchronize()
    assert netcsum.last_launch().startswith("crc_ilv_kernel<w11> G=8 ")
    smp = np.sort(np.random.default_rng(9).choice(n, size=4096, replace=False))
    rows = buf[: n * S].view(n, S)[torch.from_numpy(smp).to(DEV)].cpu().numpy()
    want = oracle.crc32_batch(rows.reshape(-1).copy(), len(smp), True, stride=S, length=L)
    assert np.array_equal(fcs.cpu().numpy().view(np.uint32)[smp], want)
    v = buf[: n * S].view(n, S)
    v[:, L:S] = fcs.view(torch.uint8).view(n, 4)
    res = torch.zeros(n, dtype=torch.int32, device=DEV)
    netcsum.crc32_strided(buf, S, S, n, res, 1)
    torch.cuda.synchronize()
    assert bool((res == RESIDUE).all())
    bad = torch.arange(0, n, 1000, device=DEV)
    v[bad, 321] ^= 0x20
    netcsum.crc32_strided(buf, S, S, n, res, 1)
    torch.cuda.synchronize()
    wrong = torch.nonzero(res != RESIDUE).flatten()
    assert torch.equal(wrong, bad)


def test_crc_varlen_every_length_and_alignment(crc_form):
    """Every length 0..700 at every start alignment mod 16 (the interleaved form's head chunk, front
    padding and tail cases; lengths < 32 take the group's sequential path)."""
    lens = np.repeat(np.arange(0, 701, dtype=np.uint32), 16)
    n = len(lens)
    off = (np.arange(n, dtype=np.uint64) * 768 + np.tile(np.arange(16, dtype=np.uint64), 701)).astype(np.uint64)
    data = np.random.default_rng(77).integers(0, 256, size=n * 768 + 64, dtype=np.uint8)
    d = torch.from_numpy(data).to(DEV)
    out = torch.zeros(n, dtype=torch.int32, device=DEV)
    netcsum.crc32_varlen(d, torch.from_numpy(off.view(np.int64)).to(DEV), torch.from_numpy(lens.view(np.int32)).to(DEV),
                         n, out, 1)
    torch.cuda.synchronize()
    assert netcsum.last_launch().startswith(expected_kernel(crc_form, 0, varlen=True)), netcsum.last_launch()
    want = oracle.crc32_batch(data, n, True, off=off, lens=lens)
    got = out.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(lens[i]), int(off[i] % 16), hex(got[i]), hex(want[i])) for i in bad[:6]]


@pytest.mark.parametrize("crc_kernel", [0, 2, 3])
def test_crc_batch_strided_empty_segments(crc_kernel):
    """len 0: every result 0 (the reference's NET_UTIL_ERR_NULL_SIZE value), nothing read."""
    netcsum.tune(netcsum.TUNE_CRC_KERNEL, crc_kernel)
    try:
        n = 5000
        d = torch.full((n * 6 + 64,), 0xAB, dtype=torch.uint8, device=DEV)
        out = torch.full((n,), -1, dtype=torch.int32, device=DEV)
        netcsum.crc32_strided(d, 6, 0, n, out, 1)
        torch.cuda.synchronize()
        assert bool((out == 0).all())
    finally:
        netcsum.tune(netcsum.TUNE_CRC_KERNEL, 0)
