"""GPU parity of the batched NET_BUF chain checksums (NetUtil_MI355X_ChkSumBatchChains) against the C
oracle walking the same pieces as NET_BUF chains (net_util.c:1545-1687), bit-exact, over every
group width, scattered odd-offset pieces, empty pieces, NULL chains, odd pseudo-headers, u32 wrap."""
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
    yield
    netcsum.tune(netcsum.TUNE_GROUP_LANES, 0)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, 0)


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


@pytest.mark.parametrize("group", [0, 16, 32, 64])
@pytest.mark.parametrize("pseudo_len", [0, 12, 13, 40])
@pytest.mark.parametrize("op", [0, 1])
def test_chain_batch_matches_oracle(group, pseudo_len, op):
    rng = random.Random(group * 131 + pseudo_len * 3 + op)
    cb = make_chain_batch(rng, 1500, pseudo_len=pseudo_len, self_verify=0.5 if op else 0.0)
    netcsum.tune(netcsum.TUNE_GROUP_LANES, group)
    got, want = _gpu(cb, op), _want(cb, op)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:5]]
    if op:
        assert 0 < int(want.sum()) < cb.n


@pytest.mark.parametrize("grid", [1, 3, 0])
def test_chain_batch_grid_stride_and_long_chains(grid):
    rng = random.Random(100 + grid)
    cb = make_chain_batch(rng, 3000, max_pieces=45, max_piece=1480, pseudo_len=12)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, grid)
    assert np.array_equal(_gpu(cb, 0), _want(cb, 0))


def test_chain_batch_u32_wrap():
    rng = random.Random(5)
    cb = make_chain_batch(rng, 64, wrap_chains=32, pseudo_len=13)
    assert np.array_equal(_gpu(cb, 0), _want(cb, 0))
    assert np.array_equal(_gpu(cb, 1), _want(cb, 1))


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
