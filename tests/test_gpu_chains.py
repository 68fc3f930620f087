"""GPU parity of the batched NET_BUF chain checksums (NetUtil_MI355X_ChkSumBatchChains) against the C
oracle walking the same pieces as NET_BUF chains (net_util.c:1545-1687), bit-exact, over every
group width, scattered odd-offset pieces, empty pieces, NULL chains, odd pseudo-headers, u32 wrap,
for the two-pass forms (per-piece sums by tiled 16-lane groups — or in the live-sector stream
with NETCSUM_TUNE_KERNEL 3 — then a combine pass per chain; NETCSUM_TUNE_KERNEL 5: one exact
half-word sum per piece from the segment live-sector stream, combined modulo 65535, chains past
128 KiB re-read exactly), the wave-per-chain form (NETCSUM_TUNE_KERNEL 1) and the two-pass forms'
fallback for batches with more pieces than their records hold."""
import random

import numpy as np
import pytest

import netcsum
import oracle
from chains import make_chain_batch

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _defaults():
    netcsum.tune(netcsum.TUNE_GROUP_LANES, 0)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, 0)
    netcsum.tune(netcsum.TUNE_KERNEL, 0)
    netcsum.tune(netcsum.TUNE_CHAIN_COMBINE, -1)
    yield
    netcsum.tune(netcsum.TUNE_CHAIN_COMBINE, -1)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, 0)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, 0)
    netcsum.tune(netcsum.TUNE_KERNEL, 0)


def _dev(a, dtype):
    return torch.from_numpy(np.ascontiguousarray(a).view(dtype)).to(DEV)


def _gpu(cb, op):
    base = _dev(cb.base, np.uint8)
    off = _dev(cb.piece_off, np.int64) if len(cb.piece_off) else torch.zeros(1, dtype=torch.int64, device=DEV)
    ln = _dev(cb.piece_len, np.int16) if len(cb.piece_len) else torch.zeros(1, dtype=torch.int16, device=DEV)
    first = _dev(cb.chain_first, np.int32)
    ph = _dev(cb.pseudo, np.uint8) if cb.pseudo is not None else None
    out = torch.zeros(cb.n, dtype=torch.int16 if op == 0 else torch.uint8, device=DEV)
    netcsum.batch_chains(base, off, ln, first, ph, cb.pseudo_stride, cb.pseudo_len, cb.n, out, op=op,
                         n_pieces=int(cb.chain_first[-1]))
    torch.cuda.synchronize()
    r = out.cpu().numpy()
    return r.view(np.uint16) if op == 0 else r


def _want(cb, op):
    return oracle.batch_chains(cb.base, cb.piece_off, cb.piece_len, cb.chain_first, cb.pseudo, cb.pseudo_stride,
                               cb.pseudo_len, cb.n, op)


# pass 1 of each TUNE_KERNEL value (0: the default)
PASS1 = {0: "seg_live_varlen_kernel", 1: "chain_wave_kernel", 3: "chain_live_piece_kernel", 4: "chain_piece_kernel",
         5: "seg_live_varlen_kernel", 6: "seg_live_varlen_kernel"}


@pytest.mark.parametrize("group", [0, 1, 3, 4, 5, 6, 16, 32, 64])  # 1-5: TUNE_KERNEL, 6: 5 with 64-lane combine,
#                                                                    16-64: TUNE_GROUP_LANES
@pytest.mark.parametrize("pseudo_len", [0, 12, 13, 40])
@pytest.mark.parametrize("op", [0, 1])
def test_chain_batch_matches_oracle(group, pseudo_len, op):
    rng = random.Random(group * 131 + pseudo_len * 3 + op)
    cb = make_chain_batch(rng, 1500, pseudo_len=pseudo_len, self_verify=0.5 if op else 0.0)
    netcsum.tune(netcsum.TUNE_CHAIN_COMBINE, 64 if group == 6 else -1)
    if group <= 6:
        netcsum.tune(netcsum.TUNE_KERNEL, 5 if group == 6 else group)
    else:
        netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    got, want = _gpu(cb, op), _want(cb, op)
    name = PASS1.get(group, "chain_batch_kernel")
    assert netcsum.last_launch().startswith(name), netcsum.last_launch()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:5]]
    if op:
        assert 0 < int(want.sum()) < cb.n


@pytest.mark.parametrize("grid", [1, 3, 0])
@pytest.mark.parametrize("kernel", [0, 1, 4])
def test_chain_batch_grid_stride_and_long_chains(grid, kernel):
    rng = random.Random(100 + grid)
    cb = make_chain_batch(rng, 3000, max_pieces=45, max_piece=1480, pseudo_len=12)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
    assert np.array_equal(_gpu(cb, 0), _want(cb, 0))


@pytest.mark.parametrize("kernel", [0, 1, 4])
def test_chain_batch_u32_wrap(kernel):
    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
    rng = random.Random(5)
    cb = make_chain_batch(rng, 64, wrap_chains=32, pseudo_len=13)
    assert np.array_equal(_gpu(cb, 0), _want(cb, 0))
    assert np.array_equal(_gpu(cb, 1), _want(cb, 1))


@pytest.mark.parametrize("kernel", [0, 4])
@pytest.mark.parametrize("n_pieces", [1, 63, 64, 65, 1000, 4097])
def test_chain_batch_piece_tiles(n_pieces, kernel):
    """Pass 1's tiles of 64 pieces (and the live stream's runs): piece counts around the tile size, one
    chain per 7 pieces."""
    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
    rng = np.random.default_rng(n_pieces)
    lens = rng.integers(0, 1600, size=n_pieces).astype(np.uint16)
    offs = np.zeros(n_pieces, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + rng.integers(0, 3, size=n_pieces - 1).astype(np.uint64))
    base = rng.integers(0, 256, size=int(offs[-1]) + 1700, dtype=np.uint8)
    first = np.minimum(np.arange(0, n_pieces + 7, 7, dtype=np.uint64), n_pieces).astype(np.uint32)
    first = np.unique(first)
    n = len(first) - 1
    ph = rng.integers(0, 256, size=12 * n, dtype=np.uint8)
    out = torch.zeros(n, dtype=torch.int16, device=DEV)
    netcsum.batch_chains(_dev(base, np.uint8), _dev(offs, np.int64), _dev(lens, np.int16), _dev(first, np.int32),
                         _dev(ph, np.uint8), 12, 12, n, out, op=0, n_pieces=n_pieces)
    torch.cuda.synchronize()
    want = oracle.batch_chains(base, offs, lens, first, ph, 12, 12, n, 0)
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)


@pytest.mark.parametrize("kernel", [0, 4])
def test_chain_batch_more_pieces_than_records(kernel):
    """The two-pass forms keep max(2^20, 128 x chains) piece records; a batch of 4 chains with
    1.2 M pieces (0-5 B each, odd lengths and addresses) is done by its wave-per-chain fallback."""
    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
    rng = np.random.default_rng(77)
    per = 300_001
    n = 4
    lens = rng.integers(0, 6, size=n * per).astype(np.uint16)
    offs = np.zeros(n * per, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + 1)                # 1-B gaps: scattered parities
    base = rng.integers(0, 256, size=int(offs[-1]) + 64, dtype=np.uint8)
    first = (np.arange(n + 1, dtype=np.uint64) * per).astype(np.uint32)
    ph = rng.integers(0, 256, size=13 * n, dtype=np.uint8)
    out = torch.zeros(n, dtype=torch.int16, device=DEV)
    netcsum.batch_chains(_dev(base, np.uint8), _dev(offs, np.int64), _dev(lens, np.int16), _dev(first, np.int32),
                         _dev(ph, np.uint8), 13, 13, n, out, op=0, n_pieces=n * per)
    torch.cuda.synchronize()
    want = oracle.batch_chains(base, offs, lens, first, ph, 13, 13, n, 0)
    assert netcsum.last_launch().startswith(PASS1[kernel])
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)


@pytest.mark.parametrize("form", [(3, 8, -1), (5, 8, 1), (5, 4, 1), (5, 8, 0), (5, 4, 0)])
@pytest.mark.parametrize("order", ["sorted", "shuffled", "far", "odd"])
@pytest.mark.parametrize("spw", [1, 7, 16, 45, 64])
def test_chain_batch_fragments_live_runs(order, spw, form):
    """Pass 1's live-sector streams on the chain row's layout — chain_live_piece_kernel (TUNE_KERNEL 3)
    and the segment stream's one-record form (TUNE_KERNEL 5; depth 4 / 8 by TUNE_CHUNKS, compacted
    sectors or not by NETCSUM_TUNE_LIVE_COMPACT): datagrams' fragments, each in its own 2-KiB buffer at
    +42 (net_ipv4.c:3963 reassembly chains), 1-45 fragments per chain, the last one short, some empty;
    runs of 1..64 pieces (TUNE_TILE). Shuffled fragments within a chain, every 5th buffer 200 KiB
    further on, or odd offsets and lengths: the runs they break take the 16-lane groups."""
    kern, depth, cmp = form
    netcsum.tune(netcsum.TUNE_KERNEL, kern)
    netcsum.tune(netcsum.TUNE_TILE, spw)
    netcsum.tune(netcsum.TUNE_CHUNKS, depth)
    netcsum.tune(netcsum.TUNE_LIVE_COMPACT, cmp)
    try:
        rng = np.random.default_rng(spw * 7 + len(order))
        per = rng.integers(1, 46, size=600)
        npc = int(per.sum())
        first = np.zeros(len(per) + 1, np.uint32)
        first[1:] = np.cumsum(per)
        lens = np.full(npc, 1480, np.uint16)
        lens[first[1:] - 1] = rng.integers(1, 1481, size=len(per))        # each chain's last fragment
        lens[rng.random(npc) < 0.02] = 0
        offs = np.arange(npc, dtype=np.uint64) * np.uint64(2048) + np.uint64(42)
        if order == "odd":
            odd = rng.random(npc) < 0.3
            offs = offs + odd.astype(np.uint64)
            lens = np.where(rng.random(npc) < 0.3, lens - (lens > 0), lens).astype(np.uint16)
        if order == "far":
            offs = offs + (np.arange(npc, dtype=np.uint64) // 5) * np.uint64(200 * 1024)
        if order == "shuffled":
            for c in range(len(per)):
                a, b = int(first[c]), int(first[c + 1])
                p = rng.permutation(b - a) + a
                offs[a:b], lens[a:b] = offs[p].copy(), lens[p].copy()
        base = rng.integers(0, 256, size=int(offs.max()) + 2048 + 64, dtype=np.uint8)
        ph = rng.integers(0, 256, size=12 * len(per), dtype=np.uint8)
        n = len(per)
        for op in (0, 1):
            out = torch.zeros(n, dtype=torch.int16 if op == 0 else torch.uint8, device=DEV)
            netcsum.batch_chains(_dev(base, np.uint8), _dev(offs, np.int64), _dev(lens, np.int16), _dev(first, np.int32),
                                 _dev(ph, np.uint8), 12, 12, n, out, op=op, n_pieces=npc)
            torch.cuda.synchronize()
            assert netcsum.last_launch().startswith(PASS1[kern]), netcsum.last_launch()
            assert f"pieces_per_wave={spw}" in netcsum.last_launch()
            if kern == 5:
                assert f"D={depth}," in netcsum.last_launch() and ("compact" in netcsum.last_launch()) == (cmp != 0)
            got = out.cpu().numpy()
            want = oracle.batch_chains(base, offs, lens, first, ph, 12, 12, n, op)
            got = got.view(np.uint16) if op == 0 else got
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (op, [(int(i), int(got[i]), int(want[i])) for i in bad[:5]])
    finally:
        netcsum.tune(netcsum.TUNE_TILE, -1)
        netcsum.tune(netcsum.TUNE_CHUNKS, 0)
        netcsum.tune(netcsum.TUNE_LIVE_COMPACT, -1)


@pytest.mark.parametrize("kernel,cl", [(0, -1), (0, 64), (4, -1), (1, -1)])
@pytest.mark.parametrize("pseudo_len", [0, 12, 13])
def test_chain_batch_mod65535_boundaries(kernel, cl, pseudo_len):
    """The one-record form's arithmetic at its edges: all-0xFF chains of 131 050 - 131 100 stream
    bytes (the modulo-65535 form up to 131 072, the exact re-read past it, the reference's u32
    accumulator at 2^32 - 1 and wrapping beyond), all-zero chains (T = 0: Calc 0xFFFF), chains whose
    sum is a positive multiple of 65535 (Calc 0), odd pieces at odd addresses; against the oracle."""
    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
    netcsum.tune(netcsum.TUNE_CHAIN_COMBINE, cl)
    rng = np.random.default_rng(pseudo_len + 3)
    chains = []                                                   # (bytes value, [piece lengths])
    for total in range(131050, 131101, 3):
        body = total - pseudo_len
        k = int(rng.integers(2, 100))
        cuts = np.sort(rng.choice(np.arange(1, body), size=k - 1, replace=False))
        ln = np.diff(np.concatenate([[0], cuts, [body]]))
        while ln.max() > 65535:
            cuts = np.sort(rng.choice(np.arange(1, body), size=k - 1, replace=False))
            ln = np.diff(np.concatenate([[0], cuts, [body]]))
        chains.append((0xFF, ln))
    for _ in range(8):
        chains.append((0x00, rng.integers(0, 1500, size=int(rng.integers(1, 9)))))
    chains.append((0xFF, np.array([2])))                          # T = 65535
    chains.append((0xFF, np.array([1, 1])))                       # T = 65535 over two odd pieces
    chains.append((0xFF, np.array([3, 3, 7, 1])))                 # T = 7 x 65535
    offs, lens, first, pos = [], [], [0], 0
    blobs = []
    for val, ln in chains:
        for L in ln:
            pos += int(rng.integers(0, 3))                        # odd and even addresses
            offs.append(pos)
            lens.append(int(L))
            blobs.append((pos, int(L), val))
            pos += int(L)
        first.append(len(offs))
    base = rng.integers(0, 256, size=pos + 64, dtype=np.uint8)
    for p, L, val in blobs:
        base[p:p + L] = val
    n = len(chains)
    ph = np.full(max(pseudo_len, 1) * n, 0xFF, np.uint8)
    ph[-pseudo_len * 11:] = 0 if pseudo_len else ph[-1:]           # the zero / multiple chains: zero pseudo
    offs, lens, first = np.array(offs, np.uint64), np.array(lens, np.uint16), np.array(first, np.uint32)
    for op in (0, 1):
        out = torch.zeros(n, dtype=torch.int16 if op == 0 else torch.uint8, device=DEV)
        netcsum.batch_chains(_dev(base, np.uint8), _dev(offs, np.int64), _dev(lens, np.int16), _dev(first, np.int32),
                             _dev(ph, np.uint8) if pseudo_len else None, pseudo_len, pseudo_len, n, out, op=op,
                             n_pieces=len(offs))
        torch.cuda.synchronize()
        assert netcsum.last_launch().startswith(PASS1[kernel]), netcsum.last_launch()
        got = out.cpu().numpy()
        got = got.view(np.uint16) if op == 0 else got
        want = oracle.batch_chains(base, offs, lens, first, ph if pseudo_len else None, pseudo_len, pseudo_len, n, op)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (op, [(int(i), int(got[i]), int(want[i])) for i in bad[:5]])
        if op == 0 and pseudo_len == 0:
            assert int(got[-4]) == 0xFFFF - 0 and all(int(g) == 0 for g in got[-3:])   # T = 0 / multiples
    netcsum.tune(netcsum.TUNE_CHAIN_COMBINE, -1)


def test_chain_batch_matches_single_segment_batch():
    """One piece per chain == the varlen segment batch on the same spans."""
    rng = random.Random(9)
    cb = make_chain_batch(rng, 2000, max_pieces=1, null_chains=0.0, empty_pieces=0.0, pseudo_len=12)
    got = _gpu(cb, 0)
    base = _dev(cb.base, np.uint8)
    out = torch.zeros(cb.n, dtype=torch.int16, device=DEV)
    netcsum.batch_varlen(base, _dev(cb.piece_off, np.int64), _dev(cb.piece_len, np.int16),
                         _dev(cb.pseudo, np.uint8), cb.pseudo_stride, 12, cb.n, out)
    torch.cuda.synchronize()
    assert np.array_equal(got, out.cpu().numpy().view(np.uint16))


@pytest.mark.parametrize("xcd,cg,touch", [(0, -1, -1), (1, -1, -1), (0, 1, -1), (1, 1, -1), (0, 3, -1),
                                           (1, -1, 1), (0, -1, 1), (16, -1, 0)])
def test_chain_pass1_tile_order(xcd, cg, touch):
    """Pass 1's XCD-aware tile order (NETCSUM_TUNE_STREAM_XCD; one tile of 64 pieces per block, the
    tiles of one XCD contiguous) and its balanced grid (NETCSUM_TUNE_CHAIN_GRID k: k x the resident
    blocks, equal contiguous shares — most blocks empty or with a few pieces at these sizes) are launch
    options, as are chunked tile orders and the row touch of a group's first pieces
    (NETCSUM_TUNE_STREAM_TOUCH): the same records, the oracle's results, for piece counts that fill the
    tiles unevenly over the 8 XCDs."""
    netcsum.tune(netcsum.TUNE_KERNEL, 4)                           # the tiled pass 1
    try:
        netcsum.tune(netcsum.TUNE_STREAM_XCD, xcd)
        netcsum.tune(netcsum.TUNE_CHAIN_GRID, cg)
        netcsum.tune(netcsum.TUNE_STREAM_TOUCH, touch)
        for n_chains, seed in ((1, 1), (37, 2), (700, 3), (3000, 4)):
            cb = make_chain_batch(random.Random(seed), n_chains, 12)
            assert np.array_equal(_gpu(cb, 0), _want(cb, 0))
            assert netcsum.last_launch().startswith("chain_piece_kernel")
    finally:
        netcsum.tune(netcsum.TUNE_STREAM_XCD, -1)
        netcsum.tune(netcsum.TUNE_CHAIN_GRID, -1)
        netcsum.tune(netcsum.TUNE_STREAM_TOUCH, -1)
