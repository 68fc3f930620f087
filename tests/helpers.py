"""Test helpers: random packet/chain generators that produce the SAME case for the C oracle, the
numpy oracle and the product library (NET_BUF ctypes chains from netcsum.Chain)."""
from __future__ import annotations

import random

import netcsum
import oracle_np as onp

PROTOS_OK = [netcsum.NET_PROTOCOL_TYPE_TCP_V4, netcsum.NET_PROTOCOL_TYPE_UDP_V4,
             netcsum.NET_PROTOCOL_TYPE_TCP_V6, netcsum.NET_PROTOCOL_TYPE_UDP_V6,
             netcsum.NET_PROTOCOL_TYPE_ICMP_V4, netcsum.NET_PROTOCOL_TYPE_ICMP_V6,
             netcsum.NET_PROTOCOL_TYPE_IP_V6_EXT_NONE]


def rand_bytes(rng: random.Random, n: int, pattern: str = "random") -> bytes:
    if pattern == "zero":
        return bytes(n)
    if pattern == "ff":
        return b"\xff" * n
    if pattern == "carry":
        return bytes((0xFF, 0xFF, 0x00, 0x01)[i & 3] for i in range(n))
    return bytes(rng.getrandbits(8) for _ in range(n))


def rand_buf(rng: random.Random, length: int, proto=None, pattern="random") -> dict:
    """A NET_BUF description whose checksummed piece has `length` bytes, placed via the fields the
    protocol type selects (net_util.c:1613-1640)."""
    proto = proto if proto is not None else rng.choice(PROTOS_OK)
    lead = rng.randint(0, 9)                         # bytes before the checksummed piece
    hdr = rng.randint(0, min(length, 60))           # split of the piece into HdrLen + DataLen
    data = rand_bytes(rng, lead + length + rng.randint(0, 5), pattern)
    b = {"data": data, "proto": proto, "offset": rng.randint(0, 7)}
    if proto in (netcsum.NET_PROTOCOL_TYPE_ICMP_V4, netcsum.NET_PROTOCOL_TYPE_ICMP_V6):
        b.update(icmp_ix=lead, icmp_hdr_len=hdr, data_len=length - hdr)
    elif proto == netcsum.NET_PROTOCOL_TYPE_IP_V6_EXT_NONE:
        b.update(tot_len=lead + length, data_len=length)
    else:
        b.update(transport_ix=lead, transport_hdr_len=hdr, data_len=length - hdr)
    return b


def to_np_buf(b: dict) -> onp.Buf:
    return onp.Buf(b["data"], proto=b["proto"], transport_ix=b.get("transport_ix", 0),
                   transport_hdr_len=b.get("transport_hdr_len", 0),
                   data_len=b.get("data_len", len(b["data"]) - b.get("transport_ix", 0)),
                   icmp_ix=b.get("icmp_ix", 0), icmp_hdr_len=b.get("icmp_hdr_len", 0),
                   tot_len=b.get("tot_len", 0))


def rand_chain(rng: random.Random, total: int, nbuf: int, pattern="random", allow_empty=True) -> list[dict]:
    """Split `total` checksummed bytes over nbuf buffers (odd splits, empty middles allowed)."""
    cuts = sorted(rng.randint(0, total) for _ in range(nbuf - 1))
    lens = [b - a for a, b in zip([0] + cuts, cuts + [total])]
    if not allow_empty:
        lens = [max(1, x) for x in lens]
    return [rand_buf(rng, ln, pattern=pattern) for ln in lens]
