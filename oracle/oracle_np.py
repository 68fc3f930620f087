"""ORACLE (second, independent restatement) — test infrastructure only.

Written from RFC 1071 and the stream view of SURVEY Appendix B, NOT from the reference's loop
structure, so that agreement with the C restatement (oracle/net_util_oracle.c, which follows
Source/net_util.c routine by routine) is evidence that both capture the reference semantics:

  1. The checksummed stream is pseudo_hdr ‖ buf_1[ix_1:ix_1+len_1] ‖ … (per-buffer (ix, len) by
     ProtocolHdrType, Source/net_util.c:1613-1640, 16-bit length arithmetic :1617,1628).
     Quirk reproduced: with pdata_buf == NULL (no buffers) a dangling odd pseudo-header octet
     is never padded in, it is dropped (it is carried into a buffer that never comes,
     net_util.c:1601-1608 then the loop at :1611 does not run).
  2. S = Σ big-endian 16-bit words of the stream (odd tail right-padded with 0x00), accumulated
     mod 2^32 (the reference's u32 `sum`, net_util.c:1554,1685).
  3. fold: while S >> 16: S = (S & 0xFFFF) + (S >> 16)   (net_util.c:1690-1692).
  4. Calc returns bswap16(~S) (host order on a little-endian CPU), Verify returns S == 0xFFFF.

Vectorised batch forms compute the same thing for N independent segments at once.
"""
from __future__ import annotations

import numpy as np

ERR_NONE = 200
ERR_NULL_SIZE = 210
ERR_INVALID_PROTOCOL = 211
ERR_NULL_PTR = 23
ERR_INVALID_IX = 622

PROTO_ICMP_V4, PROTO_ICMP_V6 = 60, 61
PROTO_UDP_V4, PROTO_TCP_V4, PROTO_UDP_V6, PROTO_TCP_V6 = 70, 71, 72, 73
PROTO_IP_V6_EXT_NONE = 48


def bswap16(v: int) -> int:
    return ((v & 0xFF) << 8) | ((v >> 8) & 0xFF)


def fold(s: int) -> int:
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def be_word_sum(stream: bytes) -> int:
    """Exact Σ of big-endian 16-bit words, odd tail padded (RFC 1071 §4.1)."""
    a = np.frombuffer(bytes(stream), dtype=np.uint8).astype(np.uint64)
    hi = int(a[0::2].sum())
    lo = int(a[1::2].sum())
    return (hi << 8) + lo


def hdr_calc(hdr: bytes) -> int:
    return bswap16((~fold(be_word_sum(hdr) & 0xFFFFFFFF)) & 0xFFFF)


def hdr_verify(hdr: bytes) -> int:
    return int(bswap16(fold(be_word_sum(hdr) & 0xFFFFFFFF)) == 0xFFFF)


class Buf:
    """A NET_BUF as the checksum sees it: protocol type, the index/length fields, data area."""

    def __init__(self, data: bytes, proto: int = PROTO_TCP_V4, transport_ix: int = 0,
                 transport_hdr_len: int = 0, data_len: int | None = None, icmp_ix: int = 0,
                 icmp_hdr_len: int = 0, tot_len: int = 0):
        self.data = bytes(data)
        self.proto = proto
        self.transport_ix = transport_ix
        self.transport_hdr_len = transport_hdr_len
        self.data_len = len(self.data) - transport_ix if data_len is None else data_len
        self.icmp_ix = icmp_ix
        self.icmp_hdr_len = icmp_hdr_len
        self.tot_len = tot_len

    def piece(self):
        """(ix, len) per net_util.c:1613-1640, or None for an unsupported protocol."""
        if self.proto in (PROTO_ICMP_V4, PROTO_ICMP_V6):
            return self.icmp_ix, (self.icmp_hdr_len + self.data_len) & 0xFFFF
        if self.proto in (PROTO_UDP_V4, PROTO_UDP_V6, PROTO_TCP_V4, PROTO_TCP_V6):
            return self.transport_ix, (self.transport_hdr_len + self.data_len) & 0xFFFF
        if self.proto == PROTO_IP_V6_EXT_NONE:
            return (self.tot_len - self.data_len) & 0xFFFF, self.data_len
        return None


def chain_stream(chain: list[Buf] | None, pseudo: bytes | None, dbg: bool = False):
    """Return (stream bytes, err)."""
    if dbg and chain is None:
        return b"", ERR_NULL_PTR
    parts = [bytes(pseudo)] if pseudo is not None else []
    bufs = chain or []
    for k, b in enumerate(bufs):
        pc = b.piece()
        if pc is None:
            return b"", ERR_INVALID_PROTOCOL
        ix, ln = pc
        if dbg and ix == 0xFFFF:
            return b"", ERR_INVALID_IX
        if dbg and k == 0 and len(bufs) == 1 and ln == 0:
            return b"", ERR_NULL_SIZE
        seg = b.data[ix:ix + ln]
        assert len(seg) == ln, "test chain reads beyond its data area"
        parts.append(seg)
    stream = b"".join(parts)
    if not bufs and pseudo is not None and len(pseudo) % 2 == 1:
        stream = stream[:-1]          # dangling pseudo octet never reaches a buffer
    return stream, ERR_NONE


def data_sum32(chain, pseudo, dbg=False):
    stream, err = chain_stream(chain, pseudo, dbg)
    if err != ERR_NONE:
        return 0, err
    return be_word_sum(stream) & 0xFFFFFFFF, ERR_NONE


def data_calc(chain, pseudo, dbg=False):
    s, err = data_sum32(chain, pseudo, dbg)
    if err != ERR_NONE:
        return 0, err
    return (~bswap16(fold(s))) & 0xFFFF, ERR_NONE


def data_verify(chain, pseudo, dbg=False):
    s, err = data_sum32(chain, pseudo, dbg)
    if err != ERR_NONE:
        return 0, err
    return int(bswap16(fold(s)) == 0xFFFF), ERR_NONE


# ---------------------------------------------------------------------------- vectorised batch
def _fold_vec(s: np.ndarray) -> np.ndarray:
    s = s.astype(np.uint64)
    for _ in range(4):
        s = (s & 0xFFFF) + (s >> 16)
    return s


def batch_rows(rows: np.ndarray, op: int) -> np.ndarray:
    """rows: (N, T) uint8, each row one complete stream (pseudo ‖ segment), equal T."""
    rows = np.asarray(rows, dtype=np.uint8)
    hi = rows[:, 0::2].astype(np.uint64).sum(axis=1)
    lo = rows[:, 1::2].astype(np.uint64).sum(axis=1)
    s = ((hi << np.uint64(8)) + lo) & np.uint64(0xFFFFFFFF)
    f = _fold_vec(s)
    host = ((f & 0xFF) << np.uint64(8)) | (f >> np.uint64(8))
    if op in (0, 2):
        return ((~host) & np.uint64(0xFFFF)).astype(np.uint16)
    return (host == 0xFFFF).astype(np.uint8)


def batch_strided(seg: np.ndarray, seg_stride: int, seg_len: int, pseudo: np.ndarray | None,
                  pseudo_stride: int, pseudo_len: int, n_seg: int, op: int = 0,
                  seg_offset: int = 0) -> np.ndarray:
    idx = seg_offset + np.arange(n_seg, dtype=np.int64)[:, None] * seg_stride + np.arange(seg_len)[None, :]
    rows = seg[idx] if seg_len else np.zeros((n_seg, 0), np.uint8)
    if pseudo is not None and pseudo_len:
        pidx = np.arange(n_seg, dtype=np.int64)[:, None] * pseudo_stride + np.arange(pseudo_len)[None, :]
        rows = np.concatenate([pseudo[pidx], rows], axis=1)
    return batch_rows(rows, op)


def batch_varlen(base: np.ndarray, seg_off, seg_len, pseudo, pseudo_stride, pseudo_len, op=0):
    out = []
    for i, (o, ln) in enumerate(zip(np.asarray(seg_off).tolist(), np.asarray(seg_len).tolist())):
        p = None
        if pseudo is not None:
            p = bytes(pseudo[i * pseudo_stride:i * pseudo_stride + pseudo_len])
        stream = (p or b"") + bytes(base[o:o + ln])
        s = be_word_sum(stream) & 0xFFFFFFFF
        h = bswap16(fold(s))
        out.append((~h) & 0xFFFF if op in (0, 2) else int(h == 0xFFFF))
    return np.array(out, dtype=np.uint16 if op in (0, 2) else np.uint8)
