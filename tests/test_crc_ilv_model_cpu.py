"""CPU model of the GPU's interleaved-chunk CRC-32 (csrc/netcsum_crc.hip, crc_ilv_kernel), checked
against the oracle restatement of net_util.c:485-636 (itself pinned to the CRC-32 check value and to
zlib in tests/test_crc_cpu.py). It restates, lane by lane, the decomposition the kernel relies on:
16-B chunks from the line below the segment start, front-padded with zero chunks to G*M, lane l
taking chunks l, l + G, ...; the register carried past the other lanes' chunks by
Z = A^(16 (G - 1)) o A^4; log2(G) merge levels with A^16 .. A^(8 G); the initial register as an xor
into the first 4 octets; the < 16 tail octets by lane G - 1. A^n is applied through four byte tables,
as the kernel's LDS tables do (built here by the reference's bit loop, net_util.c:510-524). No device
work: this pins the arithmetic, the GPU tests (tests/test_gpu_crc.py) pin the kernel."""
import random

import pytest

import oracle

POLY = 0xEDB88320


def _zero_octet(c):
    for _ in range(8):
        c = (c >> 1) ^ POLY if c & 1 else c >> 1
    return c


def _tables(n_octets):
    """S[k][b] = A^n(b << 8k): the register advanced over n zero octets."""
    t = []
    for k in range(4):
        row = []
        for b in range(256):
            c = b << (8 * k)
            for _ in range(n_octets):
                c = _zero_octet(c)
            row.append(c)
        t.append(row)
    return t


def _apply(S, c):
    return S[0][c & 0xFF] ^ S[1][(c >> 8) & 0xFF] ^ S[2][(c >> 16) & 0xFF] ^ S[3][c >> 24]


_CACHE = {}


def _set(n):
    if n not in _CACHE:
        _CACHE[n] = _tables(n)
    return _CACHE[n]


def _dword_mask(lo, hi, base):
    lo_, hi_ = min(max(lo - base, 0), 4), min(max(hi - base, 0), 4)
    mh = 0xFFFFFFFF if hi_ >= 4 else (1 << (8 * hi_)) - 1
    ml = 0 if lo_ >= 4 else (0xFFFFFFFF << (8 * lo_)) & 0xFFFFFFFF
    return mh & ml


def crc_ilv_model(mem: bytes, a: int, length: int, G: int) -> int:
    """CalcCpl of mem[a:a+length] (length >= 32) the way crc_ilv_kernel<G> computes it."""
    T, Z = _set(4), _set(4 + 16 * (G - 1))
    fs, e = a & ~15, a + length
    ce = e & ~15
    r, kc = e - ce, (ce - fs) >> 4
    m_n = (kc + G - 1) // G
    pad, lead = m_n * G - kc, a - fs
    regs = []
    for lane in range(G):
        c = 0
        for m in range(m_n):
            q = lane + G * m - pad
            if q < 0:
                continue                                   # leading zero chunks: the register stays 0
            w = [int.from_bytes(mem[fs + 16 * q + 4 * j: fs + 16 * q + 4 * j + 4], "little") for j in range(4)]
            if q in (0, 1):                                # head chunk: mask below the start, xor the init
                s = lead - 16 * q
                for j in range(4):
                    keep = _dword_mask(lead, 16, 4 * j) if q == 0 else 0xFFFFFFFF
                    w[j] = (w[j] & keep) ^ _dword_mask(s, s + 4, 4 * j)
            for j in range(3):
                c = _apply(T, c ^ w[j])
            c = _apply(T if m == m_n - 1 else Z, c ^ w[3])
        regs.append(c)
    d = 1
    while d < G:                                           # lane j % 2d == 2d - 1 takes A^(16 d)(c[j - d])
        S = _set(16 * d)
        regs = [regs[j] ^ _apply(S, regs[j - d]) if (j & (2 * d - 1)) == 2 * d - 1 else regs[j] for j in range(G)]
        d *= 2
    c = regs[G - 1]
    for k in range(r):                                     # tail octets: the reference's byte step
        c = _set(4)[3][(c ^ mem[ce + k]) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


@pytest.mark.parametrize("G", [1, 2, 4, 8, 16])
def test_interleaved_model_equals_oracle(G):
    rng = random.Random(100 + G)
    mem = bytes(rng.getrandbits(8) for _ in range(12000))
    lengths = [32, 33, 47, 48, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 1500, 1514, 4111]
    for L in lengths + [rng.randrange(32, 3000) for _ in range(6)]:
        for a in (16, 17, 18, 19, 20, 28, 29, 31):
            want, err = oracle.crc32_calc(mem[a:a + L], cpl=True)
            assert err == 200
            assert crc_ilv_model(mem, a, L, G) == want, (G, L, a % 16)


def test_compile_time_shift_tables_compose():
    """The kernel's Z and merge tables are compositions of the A^4 tables (make_tabs in
    netcsum_crc.hip composes them the same way): A^(m + n) = A^m o A^n on random registers."""
    rng = random.Random(3)
    for m, n in ((4, 4), (16, 16), (32, 32), (64, 64), (48, 4), (240, 4)):
        Sm, Sn, Smn = _set(m), _set(n), _set(m + n)
        for _ in range(64):
            c = rng.getrandbits(32)
            assert _apply(Smn, c) == _apply(Sm, _apply(Sn, c)), (m, n)
    assert _set(4)[3][1] == 0x77073096 and _set(4)[3][255] == 0x2D02EF8D   # the byte table
