"""GPU parity: every product entry point, through the C ABI, against the oracle on the same bytes.

Bar: bit-exact (integer checksums). Small/medium sizes compare every output with the C oracle
(which the KAT and cross tests pin); the full BASELINE size (config C2: 1 M x 1500 B + 12 B
pseudo-header) is checked with size-independent properties (Calc -> write back -> Verify round
trip over every segment, single-byte corruption detection) plus an oracle-compared random sample.
"""
import ctypes
import random

import numpy as np
import pytest

import netcsum
import oracle
from helpers import rand_buf, rand_bytes, rand_chain

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda"


def _reset_tuning():
    for k in (netcsum.TUNE_GRID_BLOCKS, netcsum.TUNE_GROUP_LANES, netcsum.TUNE_BLOCK_THREADS,
              netcsum.TUNE_KERNEL, netcsum.TUNE_CHUNKS, netcsum.TUNE_GRID_MULT):
        netcsum.tune(k, 0)
    netcsum.tune(netcsum.TUNE_NT_LOADS, -1)
    netcsum.tune(netcsum.TUNE_TILE, -1)
    netcsum.tune(netcsum.TUNE_STREAM_WAVES, -1)
    netcsum.tune(netcsum.TUNE_STREAM_TOUCH, -1)
    netcsum.tune(netcsum.TUNE_STREAM_XCD, -1)
    netcsum.tune(netcsum.TUNE_STORE_GATHER, -1)


@pytest.fixture(autouse=True)
def _tuning_defaults():
    _reset_tuning()
    yield
    _reset_tuning()


def _host_bytes(rng, n, pattern):
    if pattern == "zero":
        return np.zeros(n, np.uint8)
    if pattern == "ff":
        return np.full(n, 0xFF, np.uint8)
    if pattern == "carry":
        return np.resize(np.array([0xFF, 0xFF, 0x00, 0x01], np.uint8), n)
    return rng.integers(0, 256, size=n, dtype=np.uint8)


def _out(n, op):
    return torch.zeros(n, dtype=torch.int16 if op in (0, 2) else torch.uint8, device=DEV)


def _np_out(t):
    a = t.cpu().numpy()
    return a.view(np.uint16) if a.dtype == np.int16 else a


def _gpu_strided(data_d, base_off, stride, L, ph_d, pstride, plen, n, op):
    out = _out(n, op)
    netcsum.batch_strided(data_d.data_ptr() + base_off, stride, L, ph_d if plen else None, pstride, plen, n, out, op)
    torch.cuda.synchronize()
    return _np_out(out)


LENGTHS = [0, 1, 2, 3, 4, 5, 7, 15, 16, 17, 19, 20, 21, 31, 33, 40, 63, 64, 65, 127, 255, 256, 257,
           1023, 1499, 1500, 1501, 4520, 8999, 9000, 16385, 65535]


@pytest.mark.parametrize("kernel", [0, 2, 4, 6])
@pytest.mark.parametrize("L", LENGTHS)
def test_strided_matrix_vs_oracle(L, kernel):
    """Every length class x stride x base misalignment x pseudo-header shape x op, per kernel form
    (0 = library default; 4 = wave-tile LDS image where it fits, 6 = segmented stream where it
    fits, else their fallback)."""
    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
    rng = np.random.default_rng(L + 11)
    n = 37 if L < 20000 else 5
    for pattern in ("random", "zero", "ff", "carry"):
        for stride in (L, L + 1, L + 3, L + 13):
            stride = max(stride, 1)
            data = _host_bytes(rng, n * stride + L + 64, pattern)
            data_d = torch.from_numpy(data).to(DEV)
            for base_off in (0, 1, 2, 3) if pattern == "random" else (0, 1):
                for plen, pstride in ((0, 0), (12, 12), (11, 13), (40, 41), (1, 1)):
                    ph = _host_bytes(rng, n * max(pstride, 1) + 64, pattern)
                    ph_d = torch.from_numpy(ph).to(DEV)
                    pofs = int(rng.integers(0, 3)) if plen else 0
                    for op in (0, 1, 2, 3):
                        if op >= 2 and plen:
                            continue
                        got = _gpu_strided(data_d, base_off, stride, L, ph_d.data_ptr() + pofs if plen else None,
                                           pstride, plen, n, op)
                        want = oracle.batch_strided(data, stride, L, ph[pofs:] if plen else None, pstride, plen, n, op,
                                                    seg_offset=base_off)
                        assert np.array_equal(got, want), (L, pattern, stride, base_off, plen, op)


@pytest.mark.parametrize("kernel", [1, 2, 3, 4])
@pytest.mark.parametrize("group", [1, 4, 8, 16, 32, 64])
@pytest.mark.parametrize("nt,chunks,tile", [(0, 0, 0), (1, 0, 3), (0, 1, 1), (1, 8, 0), (1, 6, 7)])
def test_every_group_width_and_load_policy(kernel, group, nt, chunks, tile):
    """Force each kernel form, lane-group width, chunks-per-pass and nt policy, with a tiny grid
    (deep grid-stride loops, multi-pass segments, pipelined stages running past the end)."""
    rng = np.random.default_rng(group * 2 + nt)
    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    netcsum.tune(netcsum.TUNE_NT_LOADS, nt)
    netcsum.tune(netcsum.TUNE_CHUNKS, chunks)
    netcsum.tune(netcsum.TUNE_TILE, tile)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, 3)
    for L, stride in ((1500, 1500), (20, 20), (4519, 4523), (77, 80), (0, 5), (1, 1)):
        n = 700
        data = rng.integers(0, 256, size=n * stride + 64, dtype=np.uint8)
        ph = rng.integers(0, 256, size=n * 12 + 16, dtype=np.uint8)
        data_d, ph_d = torch.from_numpy(data).to(DEV), torch.from_numpy(ph).to(DEV)
        for op in (0, 1):
            got = _gpu_strided(data_d, 1, stride, L, ph_d.data_ptr(), 12, 12, n, op)
            want = oracle.batch_strided(data, stride, L, ph, 12, 12, n, op, seg_offset=1)
            assert np.array_equal(got, want), (kernel, group, nt, chunks, tile, L, op)
    # variable-length + long pseudo-header (> 16*G-15 B exercises the extra pseudo pass)
    base, off, lens, _ = _packed_udp(rng, 300, 0, 3000)
    ph = rng.integers(0, 256, size=300 * 1100 + 64, dtype=np.uint8)
    b_d, o_d = torch.from_numpy(base).to(DEV), torch.from_numpy(off.view(np.int64)).to(DEV)
    l_d, p_d = torch.from_numpy(lens.view(np.int16)).to(DEV), torch.from_numpy(ph).to(DEV)
    for plen, pst in ((1033, 1100), (40, 41)):
        out = _out(300, 0)
        netcsum.batch_varlen(b_d, o_d, l_d, p_d.data_ptr() + 3, pst, plen, 300, out, 0)
        torch.cuda.synchronize()
        want = oracle.batch_varlen(base, off, lens, ph[3:], pst, plen, 0)
        assert np.array_equal(_np_out(out), want), (kernel, group, plen)


def _packed_udp(rng, n, lo=40, hi=9000, pattern="random"):
    lens = rng.integers(lo, hi + 1, size=n).astype(np.uint16)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    base = _host_bytes(rng, int(off[-1]) + int(lens[-1]) + 64, pattern)
    ph = np.zeros((n, 12), np.uint8)
    ph[:, 0:4] = rng.integers(0, 256, size=(n, 4))
    ph[:, 4:8] = rng.integers(0, 256, size=(n, 4))
    ph[:, 9] = 17
    ph[:, 10] = (lens >> 8).astype(np.uint8)
    ph[:, 11] = (lens & 0xFF).astype(np.uint8)
    return base, off, lens, ph.reshape(-1).copy()


@pytest.mark.parametrize("pattern", ["random", "zero", "ff", "carry"])
def test_varlen_packed_odd_starts_vs_oracle(pattern):
    rng = np.random.default_rng(7)
    n = 3000
    base, off, lens, ph = _packed_udp(rng, n, pattern=pattern)
    assert (off & 1).sum() > n // 4                            # plenty of odd starts
    base_d, off_d = torch.from_numpy(base).to(DEV), torch.from_numpy(off.view(np.int64)).to(DEV)
    len_d, ph_d = torch.from_numpy(lens.view(np.int16)).to(DEV), torch.from_numpy(ph).to(DEV)
    for op in (0, 1):
        out = _out(n, op)
        netcsum.batch_varlen(base_d, off_d, len_d, ph_d, 12, 12, n, out, op)
        torch.cuda.synchronize()
        want = oracle.batch_varlen(base, off, lens, ph, 12, 12, op)
        assert np.array_equal(_np_out(out), want), op
    # HDR ops on variable-length spans without pseudo-header; also zero-length segments
    lens2 = lens.copy()
    lens2[::17] = 0
    len2_d = torch.from_numpy(lens2.view(np.int16)).to(DEV)
    for op in (2, 3):
        out = _out(n, op)
        netcsum.batch_varlen(base_d, off_d, len2_d, None, 0, 0, n, out, op)
        torch.cuda.synchronize()
        want = oracle.batch_varlen(base, off, lens2, None, 0, 0, op)
        assert np.array_equal(_np_out(out), want), op


def test_many_tiny_ipv4_headers_vs_oracle():
    """Config C3 shape (20-B IPv4 headers, HdrCalc semantics) at 1 M headers."""
    rng = np.random.default_rng(3)
    n = 1 << 20
    hdr = rng.integers(0, 256, size=n * 20, dtype=np.uint8)
    hdr_d = torch.from_numpy(hdr).to(DEV)
    for op in (2, 3):
        got = _gpu_strided(hdr_d, 0, 20, 20, None, 0, 0, n, op)
        want = oracle.batch_strided(hdr, 20, 20, None, 0, 0, n, op, n_threads=8)
        assert np.array_equal(got, want), op
    # write each header's checksum into bytes 10-11 -> every header verifies
    csum = _gpu_strided(hdr_d, 0, 20, 20, None, 0, 0, n, 2)
    h2 = hdr.reshape(n, 20).copy()
    h2[:, 10:12] = 0
    h2d = torch.from_numpy(h2.reshape(-1)).to(DEV)
    c0 = _gpu_strided(h2d, 0, 20, 20, None, 0, 0, n, 2)
    h2[:, 10:12] = c0.view(np.uint8).reshape(n, 2)
    ok = _gpu_strided(torch.from_numpy(h2.reshape(-1)).to(DEV), 0, 20, 20, None, 0, 0, n, 3)
    assert ok.all()
    del csum


def test_reference_signatures_on_gpu_vs_oracle():
    """The four drop-in functions (NET_BUF chains in host memory) against the C oracle."""
    rng = random.Random(99)
    for it in range(400):
        nbuf = rng.randint(1, 4)
        pat = rng.choice(["random", "random", "zero", "ff", "carry"])
        chain = rand_chain(rng, rng.choice([0, 1, 7, rng.randint(0, 3000)]), nbuf, pattern=pat)
        ch = netcsum.Chain(chain)
        plen = rng.choice([0, 11, 12, 40])
        ph = netcsum.HostBytes(rand_bytes(rng, plen, pat), rng.randint(0, 3)) if rng.random() < 0.85 else None
        args = (ch.ptr, ph.ptr if ph else None, plen if ph else 0)
        assert netcsum.DataCalc(*args) == oracle.data_calc(*args), it
        assert netcsum.DataVerify(*args) == oracle.data_verify(*args), it
        hsz = rng.randint(0, 60)
        hb = netcsum.HostBytes(rand_bytes(rng, hsz, pat), rng.randint(0, 7))
        assert netcsum.HdrCalc(hb.ptr, hsz) == oracle.hdr_calc(hb.ptr, hsz), it
        assert netcsum.HdrVerify(hb.ptr, hsz) == oracle.hdr_verify(hb.ptr, hsz), it
    # KATs straight through the drop-in
    ip = netcsum.HostBytes(bytes.fromhex("450000730000400040110000c0a80001c0a800c7"), 1)
    assert netcsum.HdrCalc(ip.ptr, 20) == (0x61B8, 200)
    bad = netcsum.Chain([{"data": b"abcd", "proto": netcsum.NET_PROTOCOL_TYPE_IGMP}])
    assert netcsum.DataCalc(bad.ptr, None, 0) == (0, 211)
    ph12 = netcsum.HostBytes(b"\x0a\x00\x00\x01\x0a\x00\x00\x02\x00\x06\x00\x14")
    assert netcsum.DataCalc(None, ph12.ptr, 12) == oracle.data_calc(None, ph12.ptr, 12)


@pytest.mark.parametrize("nbuf", [63, 64, 65, 120, 200, 1000])
def test_reference_signatures_long_chains_vs_oracle(nbuf):
    """DataCalc / DataVerify through the drop-in on NET_BUF chains longer than any fixed span
    array (net_util.c:1611-1687 has no bound; a 64 KiB datagram reassembled from 576-B-MTU
    fragments is ~120 buffers, net_ipv4.c:6523): odd splits, zero-length middles, odd and even
    pseudo-headers, and a self-verifying chain, all against the C oracle."""
    rng = random.Random(7000 + nbuf)
    for it in range(4):
        pat = ["random", "ff", "carry", "random"][it]
        chain = []
        for i in range(nbuf):
            ln = 0 if i % 13 == 6 else rng.choice([1, 2, 3, rng.randint(1, 576)])
            chain.append(rand_buf(rng, ln, pattern=pat) | {"offset": rng.randint(0, 3)})
        plen = [12, 11, 40, 1][it]
        ph = netcsum.HostBytes(rand_bytes(rng, plen, pat), rng.randint(0, 3))
        ch = netcsum.Chain(chain)
        args = (ch.ptr, ph.ptr, plen)
        c = netcsum.DataCalc(*args)
        assert c == oracle.data_calc(*args), (nbuf, it)
        assert c[1] == 200
        assert netcsum.DataVerify(*args) == oracle.data_verify(*args), (nbuf, it)
        assert netcsum.DataCalc(ch.ptr, None, 0) == oracle.data_calc(ch.ptr, None, 0), (nbuf, it)


def test_stream_sum32_reproduces_u32_wrap():
    chain = [{"data": b"\xff" * 65535, "proto": netcsum.NET_PROTOCOL_TYPE_TCP_V4} for _ in range(3)]
    ch = netcsum.Chain(chain)
    spans, err = netcsum.chain_to_spans(ch.ptr, None, 0)
    s, err2 = netcsum.stream_sum32(spans)
    want, werr = oracle.data_sum32(ch.ptr, None, 0)
    assert (s, err2) == (want, 200)
    assert netcsum.DataCalc(ch.ptr, None, 0) == oracle.data_calc(ch.ptr, None, 0)


def test_fill_matches_host_regeneration():
    n = (1 << 20) + 13
    buf = torch.empty(n + 3, dtype=torch.uint8, device=DEV)
    for pattern in range(4):
        netcsum.fill(buf, n, 0x5EED0001, pattern)
        torch.cuda.synchronize()
        got = buf[:n].cpu().numpy()
        assert np.array_equal(got[:4096], oracle.fill(0, 4096, 0x5EED0001, pattern))
        assert np.array_equal(got[n - 777:], oracle.fill(n - 777, 777, 0x5EED0001, pattern))


@pytest.mark.parametrize("probe", [0, 1, 2])
def test_read_stream_probe_runs(probe):
    buf = torch.ones((1 << 24) + 4096, dtype=torch.uint8, device=DEV)
    sink = torch.zeros(1, dtype=torch.int64, device=DEV)
    netcsum.tune(netcsum.TUNE_PROBE, probe)
    try:
        for n in (1 << 24, (1 << 24) + 4096 - 16, 16):          # whole runs, a short last run, one chunk
            netcsum.read_stream(buf, n, sink)
        torch.cuda.synchronize()
    finally:
        netcsum.tune(netcsum.TUNE_PROBE, 1)
    assert int(sink.item()) == 0


def test_host_memory_pipeline_vs_oracle():
    rng = np.random.default_rng(5)
    n, L = 50_000, 1500
    data = torch.from_numpy(rng.integers(0, 256, size=n * L, dtype=np.uint8)).pin_memory()
    ph = torch.from_numpy(rng.integers(0, 256, size=n * 12, dtype=np.uint8)).pin_memory()
    for op, chunks in ((0, 1), (0, 7), (1, 5)):
        out = torch.zeros(n, dtype=torch.int16 if op == 0 else torch.uint8).pin_memory()
        netcsum.batch_strided_host(data, L, L, ph, 12, 12, n, out, op, n_chunks=chunks)
        want = oracle.batch_strided(data.numpy(), L, L, ph.numpy(), 12, 12, n, op, n_threads=8)
        got = out.numpy().view(np.uint16) if op == 0 else out.numpy()
        assert np.array_equal(got, want), (op, chunks)


def _c2_batch(n):
    """Config C2 synthetic batch on device: n x 1500-B TCP segments + n x 12-B pseudo-headers."""
    L = 1500
    seg = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    netcsum.fill(seg, seg.numel(), 0x5EED0001, 0)
    idx = torch.arange(n, device=DEV, dtype=torch.int64)
    ph = torch.zeros(n, 12, dtype=torch.uint8, device=DEV)
    for b in range(4):
        ph[:, b] = ((idx >> (8 * (3 - b))) & 0xFF).to(torch.uint8) | 0x0A * (b == 0)
        ph[:, 4 + b] = ((idx * 7 >> (8 * (3 - b))) & 0xFF).to(torch.uint8)
    ph[:, 9] = 6
    ph[:, 10] = L >> 8
    ph[:, 11] = L & 0xFF
    torch.cuda.synchronize()
    return seg, ph.reshape(-1).contiguous(), L


def test_full_size_c2_round_trip_and_sample():
    n = 1 << 20
    seg, ph, L = _c2_batch(n)
    csum = _out(n, 0)
    netcsum.batch_strided(seg, L, L, ph, 12, 12, n, csum, 0)
    torch.cuda.synchronize()
    # sampled oracle comparison on host copies
    rng = np.random.default_rng(1)
    sample = np.sort(rng.choice(n, size=4096, replace=False))
    segs = seg.view(n, L)[torch.from_numpy(sample).to(DEV)].cpu().numpy().reshape(-1)
    phs = ph.view(n, 12)[torch.from_numpy(sample).to(DEV)].cpu().numpy().reshape(-1)
    want = oracle.batch_strided(segs, L, L, phs, 12, 12, len(sample), 0)
    assert np.array_equal(_np_out(csum)[sample], want)
    # Tx -> Rx round trip: zero the TCP checksum field (bytes 16-17), compute, store, verify all
    s2 = seg.view(n, L)
    s2[:, 16:18] = 0
    netcsum.batch_strided(seg, L, L, ph, 12, 12, n, csum, 0)
    s2[:, 16:18] = csum.view(torch.uint8).view(n, 2)
    ok = _out(n, 1)
    netcsum.batch_strided(seg, L, L, ph, 12, 12, n, ok, 1)
    torch.cuda.synchronize()
    assert bool(ok.all())
    # corrupt one byte in every 1000th segment -> exactly those fail
    bad = torch.arange(0, n, 1000, device=DEV)
    s2[bad, 700] ^= 0x5A
    netcsum.batch_strided(seg, L, L, ph, 12, 12, n, ok, 1)
    torch.cuda.synchronize()
    failed = torch.nonzero(ok == 0).flatten()
    assert torch.equal(failed, bad)


@pytest.mark.parametrize("L", list(range(1, 65)))
def test_small_aligned_kernel_vs_oracle(L):
    """seg_small_kernel (kernel 5) and seg_hdr_kernel (kernel 7, LDS-image tiles; strides <= 64 B)
    for strided, pseudo-less, 4-B-aligned segments of
    1..64 B — the C3 header shape): every length, several 4-B-aligned strides and base offsets,
    tile / grid-stride geometry, all four ops, half of the segments carrying a valid checksum
    (HdrCalc written at bytes 10-11 as in an IPv4 header) so Verify sees both verdicts."""
    rng = np.random.default_rng(1000 + L)
    n = 1025
    for stride in sorted({(L + 3) & ~3, ((L + 3) & ~3) + 4, ((L + 3) & ~3) + 64}):
        for pattern in ("random", "zero", "ff"):
            data = _host_bytes(rng, n * stride + 128, pattern)
            if L >= 12 and pattern == "random":
                for i in range(0, n, 2):
                    h = data[4 + i * stride: 4 + i * stride + L].copy()
                    h[10:12] = 0
                    c = oracle.batch_strided(h, L, L, None, 0, 0, 1, 2)[0]
                    data[4 + i * stride + 10: 4 + i * stride + 12] = np.frombuffer(np.uint16(c).tobytes(), np.uint8)
            data_d = torch.from_numpy(data).to(DEV)
            for base_off in (0, 4):
                for kernel, tile, grid, chunks in ((0, -1, 0, 0), (5, 0, 1, 0), (5, 0, 3, 0), (5, 1, 0, 0),
                                                   (5, 7, 0, 0), (5, 2, 3, 0), (7, -1, 0, 0), (7, -1, 1, 2),
                                                   (7, -1, 3, 3), (7, -1, 2, 4), (7, 1, 0, 0), (7, 1, 3, 4),
                                                   (7, 4, 0, 2), (7, 4, 2, 3), (7, 2, 5, 3)):
                    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
                    netcsum.tune(netcsum.TUNE_TILE, tile)
                    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
                    netcsum.tune(netcsum.TUNE_CHUNKS, chunks)
                    for op in (0, 1, 2, 3):
                        got = _gpu_strided(data_d, base_off, stride, L, None, 0, 0, n, op)
                        want = oracle.batch_strided(data, stride, L, None, 0, 0, n, op, seg_offset=base_off)
                        assert np.array_equal(got, want), (L, stride, pattern, base_off, kernel, tile, grid, chunks, op)
                        if kernel in (5, 7) and op == 2:
                            name = "seg_small_kernel" if kernel == 5 or stride > 64 else "seg_hdr_kernel"
                            assert netcsum.last_launch().startswith(name), netcsum.last_launch()
                    if L >= 12 and pattern == "random" and base_off == 4:
                        assert int(want.sum()) > 0                 # op 3: some headers verify
    # outside its domain kernel 5 falls back to the general form (pseudo-header, odd base)
    netcsum.tune(netcsum.TUNE_KERNEL, 5)
    data = _host_bytes(rng, 300 * 64 + 128, "random")
    data_d = torch.from_numpy(data).to(DEV)
    got = _gpu_strided(data_d, 1, 64, L, None, 0, 0, 300, 0)
    assert np.array_equal(got, oracle.batch_strided(data, 64, L, None, 0, 0, 300, 0, seg_offset=1))
    assert netcsum.last_launch().startswith("seg_pipe_kernel")


STREAM_LENGTHS = [256, 257, 300, 1023, 1024, 1025, 1499, 1500, 1501, 2048, 4520, 9000, 65535]


@pytest.mark.parametrize("L", STREAM_LENGTHS)
def test_stream_kernel_runs_vs_oracle(L):
    """seg_stream_kernel (kernel 6): a wave walks a contiguous RUN of segments (forced small grids
    make runs of 1..hundreds of segments), so segment boundaries fall at every piece / chunk / byte
    position, next to pseudo-headers of every shape and alignment, with gaps of 0..64 B."""
    rng = np.random.default_rng(L * 7 + 1)
    n = 300 if L <= 9000 else 9
    for pattern in ("random", "zero", "ff", "carry"):
        for stride in (L, L + 1, L + 3, L + 13, L + 64):
            data = _host_bytes(rng, n * stride + L + 64, pattern)
            data_d = torch.from_numpy(data).to(DEV)
            for base_off in ((0, 1, 2, 3, 5, 127) if pattern == "random" else (0, 1)):
                for plen, pstride in ((0, 0), (12, 12), (11, 13), (40, 41), (1, 1), (64, 64), (12, 0)):
                    ph = _host_bytes(rng, n * max(pstride, 1) + 128, pattern)
                    ph_d = torch.from_numpy(ph).to(DEV)
                    pofs = int(rng.integers(0, 5)) if plen else 0
                    for grid, chunks, run in ((1, 4, -1), (2, 6, -1), (3, 8, -1), (0, 0, -1), (0, 4, 1), (0, 6, 7),
                                              (0, 8, 128)):
                        netcsum.tune(netcsum.TUNE_KERNEL, 6)
                        netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
                        netcsum.tune(netcsum.TUNE_CHUNKS, chunks)
                        netcsum.tune(netcsum.TUNE_TILE, run)
                        for op in (0, 1) if plen else (0, 1, 2, 3):
                            got = _gpu_strided(data_d, base_off, stride, L, ph_d.data_ptr() + pofs if plen else None,
                                               pstride, plen, n, op)
                            assert netcsum.last_launch().startswith("seg_stream_kernel"), netcsum.last_launch()
                            want = oracle.batch_strided(data, stride, L, ph[pofs:] if plen else None, pstride, plen,
                                                        n, op, seg_offset=base_off)
                            assert np.array_equal(got, want), (L, pattern, stride, base_off, plen, pstride, grid, chunks, run, op)
    # outside its domain kernel 6 falls back to the general form
    netcsum.tune(netcsum.TUNE_KERNEL, 6)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, 0)
    netcsum.tune(netcsum.TUNE_TILE, -1)
    data = _host_bytes(rng, 40 * 200, "random")
    got = _gpu_strided(torch.from_numpy(data).to(DEV), 0, 200, 100, None, 0, 0, 40, 0)
    assert np.array_equal(got, oracle.batch_strided(data, 200, 100, None, 0, 0, 40, 0))
    assert netcsum.last_launch().startswith("seg_pipe_kernel")


def test_stream_kernel_full_c2_equals_pipe_kernel():
    """C2 at full size: the stream kernel's 1 M checksums equal the pipelined kernel's, and every
    segment verifies after write-back (size-independent round trip)."""
    n = 1 << 20
    seg, ph, L = _c2_batch(n)
    outs = []
    for kernel in (2, 0):                      # 0: the library default for C2 is the stream kernel
        netcsum.tune(netcsum.TUNE_KERNEL, kernel)
        o = _out(n, 0)
        netcsum.batch_strided(seg, L, L, ph, 12, 12, n, o, 0)
        torch.cuda.synchronize()
        outs.append(o)
    assert netcsum.last_launch().startswith("seg_stream_kernel")
    assert torch.equal(outs[0], outs[1])
    s2 = seg.view(n, L)
    s2[:, 16:18] = 0
    netcsum.batch_strided(seg, L, L, ph, 12, 12, n, outs[1], 0)
    s2[:, 16:18] = outs[1].view(torch.uint8).view(n, 2)
    ok = _out(n, 1)
    netcsum.batch_strided(seg, L, L, ph, 12, 12, n, ok, 1)
    torch.cuda.synchronize()
    assert bool(ok.all())


@pytest.mark.parametrize("L,run", [(1024, 20), (2048, 10), (4096, 5), (8192, 3), (9000, 2), (1500, 16),
                                   (1460, 16), (16384, 1)])
def test_dense_run_length_by_bytes(L, run):
    """Dense strided batches take runs of 16 segments unless that run's bytes are a multiple of 16 KiB
    or past 48 KiB; then runs of about 20 KiB that are not (profiles/r6zq_seglen.jsonl). Batches big
    enough that the small-batch halving leaves the run alone, every result against the oracle, odd and
    even bases."""
    rng = np.random.default_rng(L)
    n = max(2048 * run, 4096)
    data = _host_bytes(rng, n * L + 64, "random")
    ph = _host_bytes(rng, n * 12 + 64, "random")
    data_d, ph_d = torch.from_numpy(data).to(DEV), torch.from_numpy(ph).to(DEV)
    for base_off in (0, 1):
        got = _gpu_strided(data_d, base_off, L, L, ph_d, 12, 12, n, 0)
        ll = netcsum.last_launch()
        assert ll.startswith("seg_stream_kernel") and ll.endswith(f"segs_per_wave={run}"), ll
        want = oracle.batch_strided(data, L, L, ph, 12, 12, n, 0, seg_offset=base_off)
        assert np.array_equal(got, want), (L, base_off)


@pytest.mark.parametrize("touch", [0, 1])
@pytest.mark.parametrize("waves", [0, 3, 5, 8])
@pytest.mark.parametrize("xcd", [0, 1, 3, 16])
def test_stream_touch_and_residency_do_not_change_results(touch, waves, xcd):
    """The row-touch prologue, the residency cap and the XCD-aware block order — slices (1) or
    chunks of 3 / 16 blocks per XCD in turn, grids with and without a partial last round —
    (NETCSUM_TUNE_STREAM_TOUCH / _WAVES / _XCD) are launch options only: dense, gapped and varlen stream batches — runs short and long enough that the touch
    covers only their first 128 pieces — give the oracle's results under every combination."""
    rng = np.random.default_rng(100 * waves + touch + 7 * xcd)
    netcsum.tune(netcsum.TUNE_STREAM_XCD, xcd)                   # XCD-aware block order: also a launch option
    netcsum.tune(netcsum.TUNE_STREAM_TOUCH, touch)
    netcsum.tune(netcsum.TUNE_STREAM_WAVES, waves)
    netcsum.tune(netcsum.TUNE_KERNEL, 6)
    for L, stride, n, run in ((1500, 1500, 4099, -1), (1500, 1500, 700, 128), (9000, 9000, 300, 128),
                              (1499, 1503, 1000, -1), (65535, 65535, 5, 4)):
        data = _host_bytes(rng, n * stride + 64, "random")
        data_d = torch.from_numpy(data).to(DEV)
        ph = _host_bytes(rng, n * 12 + 64, "random")
        ph_d = torch.from_numpy(ph).to(DEV)
        netcsum.tune(netcsum.TUNE_TILE, run)
        for base_off in (0, 1):
            got = _gpu_strided(data_d, base_off, stride, L, ph_d, 12, 12, n, 0)
            assert netcsum.last_launch().startswith("seg_stream_kernel"), netcsum.last_launch()
            want = oracle.batch_strided(data, stride, L, ph, 12, 12, n, 0, seg_offset=base_off)
            assert np.array_equal(got, want), (L, stride, n, run, base_off)
    lens, off, base = None, None, None
    n = 2000
    lens = rng.integers(40, 9001, size=n).astype(np.uint16)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    base = _host_bytes(rng, int(off[-1]) + int(lens[-1]) + 64, "random")
    ph = _host_bytes(rng, n * 12 + 64, "random")
    base_d, ph_d = torch.from_numpy(base).to(DEV), torch.from_numpy(ph).to(DEV)
    off_d, len_d = torch.from_numpy(off.view(np.int64)).to(DEV), torch.from_numpy(lens.view(np.int16)).to(DEV)
    for run in (-1, 128):
        netcsum.tune(netcsum.TUNE_TILE, run)
        out = _out(n, 1)
        netcsum.batch_varlen(base_d, off_d, len_d, ph_d, 12, 12, n, out, 1)
        torch.cuda.synchronize()
        ll = netcsum.last_launch()                     # (or a stale plan's pipe form, launch_batch)
        assert ll.startswith("seg_stream_varlen_kernel") or "plan=pool" in ll, ll
        assert np.array_equal(_np_out(out), oracle.batch_varlen(base, off, lens, ph, 12, 12, 1)), run


@pytest.mark.parametrize("layout", ["packed", "packed_zero_len", "gaps", "reversed", "overlap", "mixed", "nic_ring",
                                    "gap_65"])
def test_stream_varlen_layouts_vs_oracle(layout):
    """Kernel 6 on offset/length descriptors: packed runs stream (segment ends from the run's
    descriptors), every other layout takes the per-segment path of the same kernel; runs of 1..128
    segments, pseudo-headers of 0/12/40 B, all four ops, against the oracle."""
    rng = np.random.default_rng(["packed", "packed_zero_len", "gaps", "reversed", "overlap", "mixed", "nic_ring",
                                 "gap_65"].index(layout))
    n = 700
    lens = rng.integers(0, 9001, size=n).astype(np.uint16)
    small = rng.random(n) < 0.3                                   # many short segments: several ends per piece
    lens[small] = rng.integers(1, 300, size=int(small.sum())).astype(np.uint16)
    if layout == "packed_zero_len":
        lens[::5] = 0
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    off += 3                                                      # odd base for every other segment
    if layout == "gaps":
        off += np.arange(n, dtype=np.uint64) * 7
    elif layout == "reversed":
        off = off[::-1].copy()
        lens = lens[::-1].copy()
        off[1:] = off[:-1]                                         # descending offsets, lengths shuffled
    elif layout == "overlap":
        off = (off // 2).astype(np.uint64)
    elif layout == "mixed":
        off[n // 2:] += 1                                          # second half shifted by one byte
    elif layout == "nic_ring":                                     # one 16 KiB ring buffer per datagram
        off = np.arange(n, dtype=np.uint64) * 16384 + 42
    elif layout == "gap_65":                                       # just past the streamed-gap limit
        off += np.arange(n, dtype=np.uint64) * 65
    tot = int((off + lens).max()) + 64
    base = _host_bytes(rng, tot, "random")
    base_d = torch.from_numpy(base).to(DEV)
    off_d = torch.from_numpy(off.view(np.int64)).to(DEV)
    len_d = torch.from_numpy(lens.view(np.int16)).to(DEV)
    for plen, pstride in ((0, 0), (12, 12), (40, 41)):
        ph = _host_bytes(rng, n * max(pstride, 1) + 64, "random")
        ph_d = torch.from_numpy(ph).to(DEV)
        for run, chunks in ((-1, 0), (1, 4), (7, 8), (64, 4), (128, 8), (65, 4)):
            netcsum.tune(netcsum.TUNE_KERNEL, 6)
            netcsum.tune(netcsum.TUNE_TILE, run)
            netcsum.tune(netcsum.TUNE_CHUNKS, chunks)
            for op in ((0, 1) if plen else (0, 1, 2, 3)):
                out = _out(n, op)
                netcsum.batch_varlen(base_d, off_d, len_d, ph_d if plen else None, pstride, plen, n, out, op)
                torch.cuda.synchronize()
                assert netcsum.last_launch().startswith("seg_stream_varlen_kernel"), netcsum.last_launch()
                want = oracle.batch_varlen(base, off, lens, ph if plen else None, pstride, plen, op)
                assert np.array_equal(_np_out(out), want), (layout, plen, run, chunks, op)


def test_sum_align32_hook_matches_reference_inner_sum():
    """NetUtil_16BitSumDataCalcAlign_32 (net_util.h:486-490): the unfolded network-order word sum the
    reference's inner loop adds (net_util.c:1407-1415), for 4-byte-aligned regions of 0..65532 B."""
    rng = random.Random(31)
    for size in [0, 4, 8, 20, 1480, 1500, 9000, 65532]:
        for pat in ("random", "ff", "carry"):
            data = rand_bytes(rng, size, pat)
            hb = netcsum.HostBytes(data)
            assert hb.ptr % 4 == 0
            want = sum(int.from_bytes(data[i:i + 2], "big") for i in range(0, size, 2)) & 0xFFFFFFFF
            assert netcsum.SumDataCalcAlign_32(hb.ptr, size) == want, (size, pat)


@pytest.mark.parametrize("run_bytes", [0, 1, 4096, 16384, 1 << 20])
def test_varlen_adaptive_runs_vs_oracle(run_bytes):
    """The varlen stream kernel's device-chosen run length (NETCSUM_TUNE_VARLEN_RUN_BYTES: 0 = fixed
    runs of 8; 1 -> the shortest run the grid covers, 3; 2^20 -> the longest, 128): every segment is
    covered exactly once whatever the sampled mean, for batches smaller and larger than the 4096
    samples, with long, short and empty segments and packed or reversed layouts."""
    rng = np.random.default_rng(run_bytes + 11)
    netcsum.tune(netcsum.TUNE_VARLEN_RUN_BYTES, run_bytes)
    try:
        for n, lo, hi in ((1, 40, 9000), (7, 0, 300), (300, 40, 1500), (5000, 40, 9000), (20000, 0, 600)):
            base, off, lens, ph = _packed_udp(rng, n, lo, hi)
            lens[::13] = 0
            if n > 1000:
                off, lens = off[::-1].copy(), lens[::-1].copy()      # not packed: the group path
            base_d, off_d = torch.from_numpy(base).to(DEV), torch.from_numpy(off.view(np.int64)).to(DEV)
            len_d, ph_d = torch.from_numpy(lens.view(np.int16)).to(DEV), torch.from_numpy(ph).to(DEV)
            for op in (0, 1):
                out = _out(n, op)
                netcsum.batch_varlen(base_d, off_d, len_d, ph_d, 12, 12, n, out, op)
                torch.cuda.synchronize()
                kern = netcsum.last_launch()
                # (a plan another batch left at the same addresses may pick the pipe form for a batch
                # or three: launch_batch)
                assert kern.startswith("seg_stream_varlen_kernel") or "plan=pool" in kern, kern
                assert ("adaptive" in kern) == (run_bytes != 0) or "plan=pool" in kern, kern
                want = oracle.batch_varlen(base, off, lens, ph, 12, 12, op)
                assert np.array_equal(_np_out(out), want), (n, op, kern)
    finally:
        netcsum.tune(netcsum.TUNE_VARLEN_RUN_BYTES, -1)


@pytest.mark.parametrize("gather", [0, 1])
@pytest.mark.parametrize("op", [0, 1])
@pytest.mark.parametrize("plen", [0, 12, 40])
def test_stream_result_gather_both_ways(gather, op, plen):
    """NETCSUM_TUNE_STORE_GATHER: the dense stream kernel's results per workgroup (4 runs) gathered in
    LDS and written whole by the workgroup's last wave, or per wave — Calc and Verify, pseudo-headers
    of 0 / 12 / 40 B (the 12-B ones added after the stream), batches that end inside a workgroup (one,
    two or three of its waves with a run, a short last run), runs of 1..128, odd bases."""
    netcsum.tune(netcsum.TUNE_STORE_GATHER, gather)
    rng = np.random.default_rng(31 * plen + 7 * op + gather)
    L = 1024
    for n, run in ((1, -1), (17, -1), (63, -1), (64, -1), (65, -1), (4099, -1), (4096 + 33, -1), (1000, 1),
                   (1000, 5), (3000, 128), (513, 128)):
        netcsum.tune(netcsum.TUNE_TILE, run)
        data = _host_bytes(rng, n * L + 64, "random")
        ph = _host_bytes(rng, n * max(plen, 1) + 64, "random")
        data_d, ph_d = torch.from_numpy(data).to(DEV), torch.from_numpy(ph).to(DEV)
        for base_off in (0, 3):
            got = _gpu_strided(data_d, base_off, L, L, ph_d, plen, plen, n, op)
            assert netcsum.last_launch().startswith("seg_stream_kernel"), netcsum.last_launch()
            want = oracle.batch_strided(data, L, L, ph if plen else None, plen, plen, n, op, seg_offset=base_off)
            assert np.array_equal(got, want), (n, run, base_off)
