"""Batched NET_BUF chain generator for the chain-batch tests: pieces scattered through one buffer at
random (odd) offsets, zero-length pieces, piece-less (pdata_buf == NULL) chains, odd pseudo-headers,
long all-0xFF chains that wrap the reference's u32 accumulator, and chains whose last piece holds
their own checksum so that DataVerify passes."""
from __future__ import annotations

import random

import numpy as np

import oracle_np as onp


class ChainBatch:
    def __init__(self, base, piece_off, piece_len, chain_first, pseudo, pseudo_stride, pseudo_len):
        self.base = base                      # uint8
        self.piece_off = piece_off            # uint64
        self.piece_len = piece_len            # uint16
        self.chain_first = chain_first        # uint32, n + 1
        self.pseudo = pseudo                  # uint8 (n * stride) or None
        self.pseudo_stride = pseudo_stride
        self.pseudo_len = pseudo_len

    @property
    def n(self) -> int:
        return len(self.chain_first) - 1

    def stream(self, i: int) -> bytes:
        p0, p1 = int(self.chain_first[i]), int(self.chain_first[i + 1])
        parts = []
        if self.pseudo is not None and self.pseudo_len:
            ph = bytes(self.pseudo[i * self.pseudo_stride:i * self.pseudo_stride + self.pseudo_len])
            if p0 == p1 and len(ph) % 2:
                ph = ph[:-1]                  # net_util.c:1601-1611, NULL chain
            parts.append(ph)
        for j in range(p0, p1):
            o, n = int(self.piece_off[j]), int(self.piece_len[j])
            parts.append(bytes(self.base[o:o + n]))
        return b"".join(parts)

    def expect(self, op: int) -> np.ndarray:
        """Stream-view restatement (oracle_np) of the per-chain result."""
        out = np.zeros(self.n, np.uint16 if op == 0 else np.uint8)
        for i in range(self.n):
            s = onp.be_word_sum(self.stream(i)) & 0xFFFFFFFF
            f = onp.bswap16(onp.fold(s))
            out[i] = (~f) & 0xFFFF if op == 0 else int(f == 0xFFFF)
        return out


def make_chain_batch(rng: random.Random, n_chains: int, max_pieces: int = 8, max_piece: int = 1600,
                     pseudo_len: int = 12, wrap_chains: int = 0, self_verify: float = 0.0,
                     null_chains: float = 0.05, empty_pieces: float = 0.1) -> ChainBatch:
    ff_len = 65535
    descs = []                                # per chain: list of ("rand", n) / ("ff", n)
    for i in range(n_chains):
        if i < wrap_chains:
            descs.append([("ff", rng.choice([ff_len, ff_len - 1, 40000]))
                          for _ in range(rng.randint(3, 40))])
            continue
        if rng.random() < null_chains:
            descs.append([])
            continue
        k = rng.randint(1, max_pieces)
        d = []
        for _ in range(k):
            if rng.random() < empty_pieces:
                d.append(("rand", 0))
            else:
                d.append(("rand", rng.choice([rng.randint(1, 64), rng.randint(1, max_piece)])))
        descs.append(d)

    # layout: one shared all-0xFF region for wrap chains, random pieces at random odd/even offsets
    buf = bytearray(rng.randint(0, 15))
    ff_off = len(buf)
    if wrap_chains:
        buf += b"\xff" * ff_len
    offs, lens, first = [], [], [0]
    csum_slots = []                            # (chain, piece index) reserved for self-verify
    order = []
    for i, d in enumerate(descs):
        for t in d:
            order.append((i, t))
    rng.shuffle(order)
    placed = {}
    for i, t in order:
        if t[0] == "rand":
            buf += bytes(rng.randint(0, 3))
            o = len(buf)
            pat = rng.random()
            if pat < 0.1:
                data = b"\xff" * t[1]
            elif pat < 0.15:
                data = bytes(t[1])
            else:
                data = rng.getrandbits(8 * t[1]).to_bytes(t[1], "little") if t[1] else b""
            buf += data
            placed.setdefault(i, []).append((o, t[1]))
        else:
            placed.setdefault(i, []).append((ff_off, t[1]))
    pseudo = None
    if pseudo_len:
        stride = pseudo_len + rng.randint(0, 5)
        pseudo = np.frombuffer(bytes(rng.getrandbits(8) for _ in range(n_chains * stride + 64)), np.uint8).copy()
    else:
        stride = 0
    for i in range(n_chains):
        for o, n in placed.get(i, []):
            offs.append(o)
            lens.append(n)
        if descs[i] and i >= wrap_chains and rng.random() < self_verify:
            csum_slots.append((i, len(offs)))
            buf += bytes(rng.randint(0, 1))
            offs.append(len(buf))
            lens.append(2)
            buf += b"\x00\x00"
        first.append(len(offs))
    buf += bytes(64)
    cb = ChainBatch(np.frombuffer(bytes(buf), np.uint8).copy(), np.array(offs, np.uint64),
                    np.array(lens, np.uint16), np.array(first, np.uint32), pseudo, stride, pseudo_len)
    # self-verifying chains: the checksum word (computed with the field zero) at an even stream position
    for i, j in csum_slots:
        s = cb.stream(i)
        if (len(s) - 2) % 2:
            continue                           # odd position: leave as a failing case
        c = _calc(s)
        o = int(cb.piece_off[j])
        cb.base[o:o + 2] = np.frombuffer(np.uint16(c).tobytes(), np.uint8)
    return cb


def _calc(stream: bytes) -> int:
    s = onp.be_word_sum(stream) & 0xFFFFFFFF
    return (~onp.bswap16(onp.fold(s))) & 0xFFFF
