"""Cross-check the two independent oracle restatements on random and adversarial cases.

C oracle (oracle/net_util_oracle.c) follows Source/net_util.c routine by routine (aligned and
octet-pair paths, 32-bit word loop, odd-octet carry between buffers). The numpy oracle
(oracle/oracle_np.py) is the RFC 1071 stream view of SURVEY Appendix B. Agreement over every
edge case the reference's code distinguishes pins the C oracle (the reference ships no vectors).
"""
import random

import numpy as np
import pytest

import netcsum
import oracle
import oracle_np as onp
from helpers import rand_buf, rand_bytes, rand_chain, to_np_buf


def _c_data(chain_desc, pseudo, pseudo_off, dbg=False, calc=True):
    ch = netcsum.Chain(chain_desc) if chain_desc is not None else None
    ph = netcsum.HostBytes(pseudo, pseudo_off) if pseudo is not None else None
    fn = oracle.data_calc if calc else oracle.data_verify
    return fn(ch.ptr if ch else None, ph.ptr if ph else None, len(pseudo) if pseudo is not None else 0, dbg)


def _np_data(chain_desc, pseudo, dbg=False, calc=True):
    bufs = [to_np_buf(b) for b in chain_desc] if chain_desc is not None else None
    fn = onp.data_calc if calc else onp.data_verify
    return fn(bufs, pseudo, dbg)


@pytest.mark.parametrize("seed", range(4))
def test_headers_1_to_60_bytes_all_offsets(seed):
    rng = random.Random(seed)
    for size in range(0, 61):
        for off in range(8):
            pat = rng.choice(["random", "random", "zero", "ff", "carry"])
            h = rand_bytes(rng, size, pat)
            hb = netcsum.HostBytes(h, off)
            assert oracle.hdr_calc(hb.ptr, size) == (onp.hdr_calc(h), 200), (size, off, pat)
            assert oracle.hdr_verify(hb.ptr, size) == (onp.hdr_verify(h), 200), (size, off, pat)


@pytest.mark.parametrize("pseudo_len", [0, 1, 11, 12, 40])
def test_single_buffer_data(pseudo_len):
    rng = random.Random(1000 + pseudo_len)
    lengths = list(range(0, 70)) + [1499, 1500, 1501, 4519, 8999, 9000, 65535] + \
        [rng.randint(1, 9000) for _ in range(60)]
    for ln in lengths:
        pat = rng.choice(["random", "random", "random", "zero", "ff", "carry"])
        b = rand_buf(rng, ln, pattern=pat)
        pseudo = rand_bytes(rng, pseudo_len, pat) if pseudo_len or rng.random() < 0.5 else None
        poff = rng.randint(0, 7)
        for calc in (True, False):
            assert _c_data([b], pseudo, poff, calc=calc) == _np_data([b], pseudo, calc=calc), (ln, pseudo_len)


@pytest.mark.parametrize("nbuf", [2, 3, 4, 6])
def test_chains_odd_splits_and_empty_buffers(nbuf):
    rng = random.Random(77 + nbuf)
    for _ in range(150):
        total = rng.choice([0, 1, 2, 3, rng.randint(0, 200), rng.randint(0, 3000)])
        pat = rng.choice(["random", "random", "zero", "ff", "carry"])
        chain = rand_chain(rng, total, nbuf, pattern=pat)
        plen = rng.choice([0, 1, 3, 11, 12, 40])
        pseudo = rand_bytes(rng, plen, pat) if rng.random() < 0.8 else None
        for calc in (True, False):
            assert _c_data(chain, pseudo, rng.randint(0, 7), calc=calc) == _np_data(chain, pseudo, calc=calc)


def test_u32_accumulator_wraps_like_the_reference():
    """Three 65535-byte all-0xFF buffers: the exact big-endian sum exceeds 2^32 and the reference's
    u32 `sum` (net_util.c:1554,1685) wraps; both oracles must reproduce the wrapped value."""
    chain = [{"data": b"\xff" * 65535, "proto": netcsum.NET_PROTOCOL_TYPE_TCP_V4} for _ in range(3)]
    ch = netcsum.Chain(chain)
    s32, err = oracle.data_sum32(ch.ptr, None, 0)
    exact = onp.be_word_sum(b"\xff" * (3 * 65535))
    assert exact > 2 ** 32 and err == 200
    assert s32 == exact & 0xFFFFFFFF
    assert onp.data_sum32([to_np_buf(b) for b in chain], None) == (s32, 200)
    assert _c_data(chain, None, 0) == _np_data(chain, None)


def test_invalid_protocol_anywhere_in_chain():
    rng = random.Random(5)
    for pos in range(3):
        chain = rand_chain(rng, 300, 3)
        chain[pos]["proto"] = rng.choice([0, 40, 62, 80])
        assert _c_data(chain, b"\x01\x02\x03", 1) == (0, 211)
        assert _np_data(chain, b"\x01\x02\x03") == (0, 211)


def test_dbg_argument_checks():
    """NET_ERR_CFG_ARG_CHK_DBG_EN = DEF_ENABLED behaviour (net_util.c:1566-1577, 1642-1672)."""
    assert oracle.data_calc(None, None, 0, dbg=True) == (0, 23)
    one_empty = [{"data": b"", "proto": netcsum.NET_PROTOCOL_TYPE_UDP_V4}]
    assert _c_data(one_empty, b"\x01" * 12, 0, dbg=True) == (0, 210)
    assert _np_data(one_empty, b"\x01" * 12, dbg=True) == (0, 210)
    assert _c_data(one_empty, b"\x01" * 12, 0, dbg=False) == _np_data(one_empty, b"\x01" * 12)
    bad_ix = [{"data": b"abcdef", "proto": netcsum.NET_PROTOCOL_TYPE_TCP_V4, "transport_ix": 0xFFFF,
               "data_len": 0, "transport_hdr_len": 0}]
    assert _c_data(bad_ix, None, 0, dbg=True) == (0, 622)
    two = [{"data": b"", "proto": 71}, {"data": b"ab", "proto": 71}]   # empty FIRST of two: fine
    assert _c_data(two, None, 0, dbg=True) == _np_data(two, None, dbg=True) != (0, 210)


def test_batch_drivers_match_np():
    rng = np.random.default_rng(3)
    n, L, stride = 257, 1500, 1503
    data = rng.integers(0, 256, size=n * stride + 16, dtype=np.uint8)
    pseudo = rng.integers(0, 256, size=n * 13, dtype=np.uint8)
    for op in range(4):
        ph = pseudo if op < 2 else None
        a = oracle.batch_strided(data, stride, L, ph, 13, 12 if op < 2 else 0, n, op, n_threads=2, seg_offset=1)
        b = onp.batch_strided(data, stride, L, ph, 13, 12 if op < 2 else 0, n, op, seg_offset=1)
        assert np.array_equal(a, b), op
    off = np.cumsum(np.r_[0, rng.integers(40, 9001, size=99)]).astype(np.uint64)
    lens = np.diff(np.r_[off, off[-1] + 500]).astype(np.uint16)
    base = rng.integers(0, 256, size=int(off[-1]) + 600, dtype=np.uint8)
    a = oracle.batch_varlen(base, off, lens, pseudo, 12, 12, 0)
    b = onp.batch_varlen(base, off, lens, pseudo, 12, 12, 0)
    assert np.array_equal(a, b)


def test_fill_patterns():
    a = oracle.fill(0, 64, 0x5EED0001, 3)
    assert bytes(a[:8]) == bytes.fromhex("ffff0001ffff0001")
    r1 = oracle.fill(0, 100, 7, 0)
    r2 = oracle.fill(37, 50, 7, 0)
    assert np.array_equal(r1[37:87], r2)
