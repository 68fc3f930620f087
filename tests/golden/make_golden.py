#!/usr/bin/env python3
"""Generate tests/golden/netutil_golden.json — small committed input/expected-output vectors for
the four reference functions (Source/net_util.c:159, :245, :344, :428).

Where the expected values come from: the reference ships no fixtures and its net_util.c cannot be
built in this image without stand-in platform headers, so the expected values
are produced by the C oracle (oracle/net_util_oracle.c) and, at generation time, asserted equal to
the independent numpy oracle (oracle/oracle_np.py). Two external KATs (RFC 1071 §3, IPv4 header)
are included with their PUBLISHED answers, not computed ones. The vectors thereby pin every later
change of either oracle or of the GPU path to today's KAT-pinned behaviour.

Coverage: KATs; HdrCalc/HdrVerify on 0..60 B at offsets 0..7; DataCalc/DataVerify on
single buffers 0..9000 B at offsets 0..7 with pseudo sizes 0/11/12/40; chains of 2..4 buffers with
odd splits and zero-length middles; ICMP / IPv6-ext-none index selection; invalid protocol;
all-zero and all-0xFF data; size-0 header; NULL chain with (odd) pseudo-header.

Run: python tests/golden/make_golden.py   (rewrites the JSON; commit it with this script)
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for sub in ("uc-tcp-ip_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, sub))

import netcsum          # noqa: E402  (ctypes NET_BUF mirror only; no device calls)
import oracle           # noqa: E402
import oracle_np as onp  # noqa: E402
from helpers import rand_buf, rand_bytes, rand_chain, to_np_buf  # noqa: E402


def hdr_case(data: bytes, offset: int, note: str = ""):
    hb = netcsum.HostBytes(data, offset)
    c, e1 = oracle.hdr_calc(hb.ptr, len(data))
    v, e2 = oracle.hdr_verify(hb.ptr, len(data))
    assert (c, v) == (onp.hdr_calc(data), onp.hdr_verify(data)) and e1 == e2 == 200
    return {"kind": "hdr", "note": note, "data": data.hex(), "offset": offset,
            "calc": c, "verify": v, "err": 200}


def data_case(chain, pseudo, pseudo_off: int, note: str = ""):
    ch = netcsum.Chain(chain) if chain is not None else None
    ph = netcsum.HostBytes(pseudo, pseudo_off) if pseudo is not None else None
    args = (ch.ptr if ch else None, ph.ptr if ph else None, len(pseudo) if pseudo is not None else 0)
    c, e1 = oracle.data_calc(*args)
    v, e2 = oracle.data_verify(*args)
    bufs = [to_np_buf(b) for b in chain] if chain is not None else None
    assert (c, e1) == onp.data_calc(bufs, pseudo) and (v, e2) == onp.data_verify(bufs, pseudo), note
    enc = None
    if chain is not None:
        enc = []
        for b in chain:
            d = dict(b)
            d["data"] = b["data"].hex()
            enc.append(d)
    return {"kind": "data", "note": note, "chain": enc, "pseudo": pseudo.hex() if pseudo is not None else None,
            "pseudo_offset": pseudo_off, "calc": c, "verify": v, "err": e1}


def main():
    rng = random.Random(0x5EED)
    cases = []
    # ---- published KATs (expected values are the published ones; asserted, not computed)
    k1 = hdr_case(bytes.fromhex("0001f203f4f5f6f7"), 0, "RFC 1071 §3 worked example: checksum bytes 22 0d")
    assert k1["calc"] == 0x0D22
    k2 = hdr_case(bytes.fromhex("450000730000400040110000c0a80001c0a800c7"), 0, "IPv4 header KAT: b861")
    assert k2["calc"] == 0x61B8
    k3 = hdr_case(bytes.fromhex("45000073000040004011b861c0a80001c0a800c7"), 2, "IPv4 KAT verify")
    assert k3["verify"] == 1
    cases += [k1, k2, k3]
    # ---- headers 0..60 at every offset
    for size in range(0, 61):
        for off in range(8):
            pat = rng.choice(["random"] * 4 + ["zero", "ff", "carry"])
            cases.append(hdr_case(rand_bytes(rng, size, pat), off, f"hdr {size}B off{off} {pat}"))
    # ---- single buffers with pseudo-headers
    lens = [0, 1, 2, 3, 19, 20, 21, 40, 63, 64, 65, 127, 1499, 1500, 1501, 4520, 8999, 9000]
    for ln in lens:
        for plen in (0, 11, 12, 40):
            pat = rng.choice(["random"] * 4 + ["zero", "ff", "carry"])
            b = rand_buf(rng, ln, pattern=pat)
            pseudo = rand_bytes(rng, plen, pat) if (plen or rng.random() < 0.5) else None
            cases.append(data_case([b], pseudo, rng.randint(0, 7), f"buf {ln}B pseudo{plen} {pat}"))
    # ---- chains
    for nbuf in (2, 3, 4):
        for _ in range(25):
            total = rng.choice([0, 1, 3, rng.randint(0, 100), rng.randint(100, 1600)])
            pat = rng.choice(["random"] * 4 + ["zero", "ff", "carry"])
            plen = rng.choice([0, 11, 12, 40])
            ch = rand_chain(rng, total, nbuf, pattern=pat)
            cases.append(data_case(ch, rand_bytes(rng, plen, pat), rng.randint(0, 7),
                                   f"chain {nbuf}x total{total} pseudo{plen} {pat}"))
    # ---- protocol index selection, invalid protocol, NULL chain
    for proto in (60, 61, 48, 70, 71, 72, 73):
        cases.append(data_case([rand_buf(rng, 77, proto=proto)], None, 0, f"proto {proto} index selection"))
    for proto in (0, 40, 62, 80):
        cases.append(data_case([{"data": b"\x12\x34\x56", "proto": proto}], b"\x01" * 12, 0, f"invalid proto {proto}"))
    cases.append(data_case(None, bytes.fromhex("c0a80001c0a800c700060014"), 0, "NULL chain, 12-B pseudo"))
    cases.append(data_case(None, bytes.fromhex("c0a80001c0a800c7000600"), 1, "NULL chain, 11-B pseudo: octet dropped"))
    out = {"generator": "tests/golden/make_golden.py", "source": "C oracle == numpy oracle; KATs published",
           "net_buf_layout": "include/netcsum_netbuf.h (template cfg, LP64)", "cases": cases}
    path = os.path.join(HERE, "netutil_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"wrote {len(cases)} cases to {path} ({os.path.getsize(path)} bytes)")


if __name__ == "__main__":
    main()
