"""GPU parity of the batched NET_BUF chain checksums (NetUtil_MI355X_ChkSumBatchChains) against the C
oracle walking the same pieces as NET_BUF chains (net_util.c:1545-1687), bit-exact, over every
group width, scattered odd-offset pieces, empty pieces, NULL chains, odd pseudo-headers, u32 wrap,
for the default two-pass form (per-piece sums, then a combine pass per chain), the wave-per-chain form
(NETCSUM_TUNE_KERNEL 1) and the two-pass form's fallback for batches with more pieces than its
records hold."""
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
    yield
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


@pytest.mark.parametrize("group", [0, 1, 16, 32, 64])           # 1: the wave-per-chain form (KERNEL 1)
@pytest.mark.parametrize("pseudo_len", [0, 12, 13, 40])
@pytest.mark.parametrize("op", [0, 1])
def test_chain_batch_matches_oracle(group, pseudo_len, op):
    rng = random.Random(group * 131 + pseudo_len * 3 + op)
    cb = make_chain_batch(rng, 1500, pseudo_len=pseudo_len, self_verify=0.5 if op else 0.0)
    if group == 1:
        netcsum.tune(netcsum.TUNE_KERNEL, 1)
    else:
        netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    got, want = _gpu(cb, op), _want(cb, op)
    assert netcsum.last_launch().startswith("chain_wave_kernel" if group == 1 else "chain_batch_kernel" if group
                                            else "chain_piece_kernel"), netcsum.last_launch()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:5]]
    if op:
        assert 0 < int(want.sum()) < cb.n


@pytest.mark.parametrize("grid", [1, 3, 0])
@pytest.mark.parametrize("kernel", [0, 1])
def test_chain_batch_grid_stride_and_long_chains(grid, kernel):
    rng = random.Random(100 + grid)
    cb = make_chain_batch(rng, 3000, max_pieces=45, max_piece=1480, pseudo_len=12)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
    assert np.array_equal(_gpu(cb, 0), _want(cb, 0))


@pytest.mark.parametrize("kernel", [0, 1])
def test_chain_batch_u32_wrap(kernel):
    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
    rng = random.Random(5)
    cb = make_chain_batch(rng, 64, wrap_chains=32, pseudo_len=13)
    assert np.array_equal(_gpu(cb, 0), _want(cb, 0))
    assert np.array_equal(_gpu(cb, 1), _want(cb, 1))


@pytest.mark.parametrize("n_pieces", [1, 63, 64, 65, 1000, 4097])
def test_chain_batch_piece_tiles(n_pieces):
    """Pass 1's tiles of 64 pieces: piece counts around the tile size, one chain per 7 pieces."""
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


def test_chain_batch_more_pieces_than_records():
    """The two-pass form keeps max(2^20, 128 x chains) piece records; a batch of 4 chains with
    1.2 M pieces (0-5 B each, odd lengths and addresses) is done by its wave-per-chain fallback."""
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
    assert netcsum.last_launch().startswith("chain_piece_kernel")
    assert np.array_equal(out.cpu().numpy().view(np.uint16), want)


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
