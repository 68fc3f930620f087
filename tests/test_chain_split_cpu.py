"""CPU model of the chain kernels' arithmetic (csrc/netcsum_chains.hip), checked against the C oracle:

* pass 1 (chain_piece_kernel) sums each piece's masked 16-B chunks as a byte sum b (v_sad_u8) and a
  little-endian half-word sum h (v_sad_u16) in the absolute, dword-aligned frame, so h = e + 256 o
  with e / o the bytes at even / odd ADDRESSES, and splits them exactly: o = (h - b) * 255^-1 mod 2^32
  (0xFEFEFEFF), e = b - o;
* pass 2 (chain_combine_kernel) gives piece j the stream parity (pseudo-header length + the lengths
  of the pieces before it) mod 2, swaps (e, o) where that differs from the piece's address parity,
  adds the pseudo-header's (e, o), and folds 256 E + O wrapped to u32 (net_util.c:1554, :1685).

The model's checksums must equal the oracle's NetUtil_16BitOnesCplChkSumDataCalc over the same
NET_BUF chains (net_util.c:1545-1687), including odd-length pieces, odd addresses, empty pieces,
NULL chains with odd pseudo-headers and chains past the u32 wrap."""
import numpy as np
import pytest

import oracle

INV255 = 0xFEFEFEFF


def split(base: np.ndarray, a: int, n: int):
    """(e, o) of base[a:a+n] by the device's route: masked aligned chunks -> (b, h) -> exact split."""
    if n == 0:
        return 0, 0
    q0, q1 = a & ~15, (a + n + 15) & ~15
    chunk = np.zeros(q1 - q0, np.uint8)
    chunk[a - q0:a - q0 + n] = base[a:a + n]
    b = int(chunk.astype(np.uint64).sum())
    h = int(chunk.view("<u2").astype(np.uint64).sum())           # v_sad_u16 of both halves of each dword
    assert h < 2 ** 32 and b < 2 ** 32
    o = ((h - b) * INV255) % 2 ** 32
    e = b - o
    seg = base[a:a + n].astype(np.int64)
    assert (e, o) == (int(seg[(np.arange(a, a + n) % 2) == 0].sum()), int(seg[(np.arange(a, a + n) % 2) == 1].sum()))
    return e, o


def model_chain(base, offs, lens, p0, p1, ph, pa, plen):
    E = O = 0
    if plen:
        pl = plen - 1 if (p0 == p1 and plen & 1) else plen           # NULL chain quirk
        e, o = split(ph, pa, pl)
        if pa & 1:
            e, o = o, e
        E, O = e, o
    par = plen & 1
    for j in range(p0, p1):
        e, o = split(base, int(offs[j]), int(lens[j]))
        if (int(offs[j]) & 1) ^ par:
            e, o = o, e
        E += e
        O += o
        par ^= int(lens[j]) & 1
    s = ((E << 8) + O) % 2 ** 32
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    host = ((s & 0xFF) << 8) | (s >> 8)
    return (~host) & 0xFFFF


@pytest.mark.parametrize("seed", range(4))
def test_split_and_combine_model_matches_oracle(seed):
    rng = np.random.default_rng(seed)
    n_pieces = 600
    lens = rng.integers(0, 2000, size=n_pieces).astype(np.uint16)
    lens[rng.random(n_pieces) < 0.1] = 0
    gaps = rng.integers(0, 5, size=n_pieces).astype(np.uint64)
    offs = np.zeros(n_pieces, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    base = rng.integers(0, 256, size=int(offs[-1]) + 2100, dtype=np.uint8)
    cuts = np.sort(rng.choice(np.arange(1, n_pieces), size=60, replace=False))
    first = np.concatenate([[0], cuts, [n_pieces]]).astype(np.uint32)
    first = np.insert(first, 5, first[5])                              # a NULL chain
    n = len(first) - 1
    plen = 13
    ph = rng.integers(0, 256, size=plen * n + 16, dtype=np.uint8)
    want = oracle.batch_chains(base, offs, lens, first, ph[: plen * n], plen, plen, n, 0)
    got = [model_chain(base, offs, lens, int(first[i]), int(first[i + 1]), ph, plen * i, plen) for i in range(n)]
    assert np.array_equal(np.array(got, np.uint16), want)


def test_split_past_the_u32_wrap():
    """A chain of 40 all-0xFF pieces of 65 534 B at odd addresses: the exact total exceeds 2^32, so
    the result depends on the reference's u32 wrap, which the model (and the kernel) reproduce."""
    per, L = 40, 65534
    base = np.full(per * (L + 1) + 32, 0xFF, np.uint8)
    offs = (np.arange(per, dtype=np.uint64) * (L + 1) + 1).astype(np.uint64)
    lens = np.full(per, L, np.uint16)
    first = np.array([0, per], np.uint32)
    ph = np.arange(12, dtype=np.uint8)
    want = oracle.batch_chains(base, offs, lens, first, ph, 12, 12, 1, 0)
    assert model_chain(base, offs, lens, 0, per, ph, 0, 12) == int(want[0])


# ---- the one-record form (round 6: seg_live_varlen_kernel<..., CH> + chain_combine_h_kernel) ----
MOD_MAX = 131072                                                      # kChainModMax


def half_word_sum(base: np.ndarray, a: int, n: int) -> int:
    """Pass 1's record: the exact little-endian half-word sum h = e + 256 o of base[a:a+n] in the
    absolute frame (the live stream's wave total of v_sad_u16 over its 128-B-aligned run)."""
    if n == 0:
        return 0
    q0, q1 = a & ~1, (a + n + 1) & ~1
    w = np.zeros(q1 - q0, np.uint8)
    w[a - q0:a - q0 + n] = base[a:a + n]
    h = int(w.view("<u2").astype(np.uint64).sum())
    assert h < 2 ** 31                                                # pieces < 64 KiB
    return h


def fold64(s: int) -> int:
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def model_chain_h(base, offs, lens, p0, p1, ph, pa, plen):
    """chain_combine_h_kernel: S = sum(swap ? h : 256 h) + the pseudo-header's 256 E + O, folded —
    T's one's-complement residue while the chain holds <= 131 072 stream bytes; longer chains take
    the exact even / odd form (model_chain)."""
    pl = (plen - 1 if (p0 == p1 and plen & 1) else plen) if plen else 0
    if pl + sum(int(lens[j]) for j in range(p0, p1)) > MOD_MAX:
        return model_chain(base, offs, lens, p0, p1, ph, pa, plen)
    S = 0
    if pl:
        e, o = split(ph, pa, pl)
        S += (o << 8) + e if pa & 1 else (e << 8) + o
    par = plen & 1
    for j in range(p0, p1):
        h = half_word_sum(base, int(offs[j]), int(lens[j]))
        S += h if (int(offs[j]) & 1) ^ par else h << 8
        par ^= int(lens[j]) & 1
    s = fold64(S)
    host = ((s & 0xFF) << 8) | (s >> 8)
    return (~host) & 0xFFFF


@pytest.mark.parametrize("seed", range(4))
def test_one_record_model_matches_oracle(seed):
    rng = np.random.default_rng(100 + seed)
    n_pieces = 600
    lens = rng.integers(0, 2000, size=n_pieces).astype(np.uint16)
    lens[rng.random(n_pieces) < 0.1] = 0
    gaps = rng.integers(0, 5, size=n_pieces).astype(np.uint64)
    offs = np.zeros(n_pieces, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gaps[:-1])
    base = rng.integers(0, 256, size=int(offs[-1]) + 2100, dtype=np.uint8)
    cuts = np.sort(rng.choice(np.arange(1, n_pieces), size=60, replace=False))
    first = np.concatenate([[0], cuts, [n_pieces]]).astype(np.uint32)
    first = np.insert(first, 5, first[5])                              # a NULL chain
    n = len(first) - 1
    plen = 13 if seed & 1 else 12
    ph = rng.integers(0, 256, size=plen * n + 16, dtype=np.uint8)
    want = oracle.batch_chains(base, offs, lens, first, ph[: plen * n], plen, plen, n, 0)
    got = [model_chain_h(base, offs, lens, int(first[i]), int(first[i + 1]), ph, plen * i, plen) for i in range(n)]
    assert np.array_equal(np.array(got, np.uint16), want)


@pytest.mark.parametrize("total", [131070, 131072, 131074, 131076])
def test_one_record_model_at_the_modulo_bound(total):
    """All-0xFF chains around the 131 072-B bound (T = 2^32 - 1 at 131 074 B, the u32 wrap beyond),
    odd pieces at odd addresses, and sums that are positive multiples of 65535 / zero."""
    rng = np.random.default_rng(total)
    k = 5
    cuts = np.sort(rng.choice(np.arange(1, total - 12), size=k - 1, replace=False))
    lens = np.diff(np.concatenate([[0], cuts, [total - 12]])).astype(np.uint16)
    offs = np.cumsum(np.concatenate([[1], lens[:-1].astype(np.uint64) + 1])).astype(np.uint64)
    base = np.full(int(offs[-1]) + int(lens[-1]) + 8, 0xFF, np.uint8)
    first = np.array([0, k], np.uint32)
    ph = np.full(12, 0xFF, np.uint8)
    want = oracle.batch_chains(base, offs, lens, first, ph, 12, 12, 1, 0)
    assert model_chain_h(base, offs, lens, 0, k, ph, 0, 12) == int(want[0])
    z = np.zeros(64, np.uint8)
    assert model_chain_h(z, np.array([1, 9], np.uint64), np.array([3, 5], np.uint16), 0, 2, z, 0, 12) == 0xFFFF
    f = np.full(64, 0xFF, np.uint8)
    assert model_chain_h(f, np.array([1, 9], np.uint64), np.array([3, 3], np.uint16), 0, 2, z, 0, 0) == 0
