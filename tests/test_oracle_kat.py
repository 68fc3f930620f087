"""Pin the oracles with the published known-answer tests (the reference ships none).

KAT 1 — RFC 1071 §3 worked example: bytes 00 01 f2 03 f4 f5 f6 f7, one's-complement sum ddf2,
        checksum bytes 22 0d (host-order return value 0x0d22 on a little-endian CPU).
KAT 2 — the classic IPv4 header 4500 0073 0000 4000 4011 0000 c0a8 0001 c0a8 00c7 with checksum
        b861 (bytes b8 61 -> return 0x61b8); re-inserted, HdrVerify returns DEF_OK.
Plus the reference-specific behaviours: all-zero data checksums to 0xFFFF
and never verifies; size-0 header -> 0xFFFF with NET_UTIL_ERR_NONE (DBG checks off); NULL chain
with a pseudo-header -> pseudo-header only; unknown protocol -> (0, 211).
"""
import pytest

import netcsum
import oracle
import oracle_np as onp

RFC1071 = bytes.fromhex("0001f203f4f5f6f7")
IPV4 = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
IPV4_OK = bytes.fromhex("45000073000040004011b861c0a80001c0a800c7")


@pytest.mark.parametrize("offset", range(8))
def test_rfc1071_example_c_oracle(offset):
    hb = netcsum.HostBytes(RFC1071, offset)
    v, err = oracle.hdr_calc(hb.ptr, hb.len)
    assert err == 200
    assert v == 0x0D22
    assert v.to_bytes(2, "little") == bytes.fromhex("220d")


def test_rfc1071_example_np_oracle():
    assert onp.be_word_sum(RFC1071) == 0x2DDF0
    assert onp.fold(0x2DDF0) == 0xDDF2
    assert onp.hdr_calc(RFC1071) == 0x0D22


@pytest.mark.parametrize("offset", range(8))
def test_ipv4_header_kat(offset):
    hb = netcsum.HostBytes(IPV4, offset)
    v, err = oracle.hdr_calc(hb.ptr, hb.len)
    assert (v, err) == (0x61B8, 200)
    assert v.to_bytes(2, "little") == bytes.fromhex("b861")
    ok = netcsum.HostBytes(IPV4_OK, offset)
    assert oracle.hdr_verify(ok.ptr, ok.len) == (1, 200)
    assert oracle.hdr_verify(hb.ptr, hb.len) == (0, 200)
    assert onp.hdr_calc(IPV4) == 0x61B8 and onp.hdr_verify(IPV4_OK) == 1


def test_ipv4_kat_as_data_path():
    """The same KAT through DataCalc: one ICMP-typed NET_BUF whose piece is the header bytes."""
    ch = netcsum.Chain([{"data": IPV4, "proto": netcsum.NET_PROTOCOL_TYPE_ICMP_V4, "icmp_ix": 0,
                         "icmp_hdr_len": 20, "data_len": 0}])
    assert oracle.data_calc(ch.ptr, None, 0) == (0x61B8, 200)


def test_all_zero_and_empty():
    z = netcsum.HostBytes(bytes(4))
    assert oracle.hdr_calc(z.ptr, 4) == (0xFFFF, 200)
    assert oracle.hdr_verify(z.ptr, 4) == (0, 200)
    assert oracle.hdr_calc(z.ptr, 0) == (0xFFFF, 200)          # DBG checks off (net_cfg.h:184)
    assert oracle.hdr_calc(z.ptr, 0, dbg=True) == (0, 210)     # net_util.c:174-178
    assert oracle.hdr_calc(None, 4, dbg=True) == (0, 23)        # net_util.c:168-172
    ff = netcsum.HostBytes(b"\xff" * 6)
    assert oracle.hdr_calc(ff.ptr, 6) == (0x0000, 200)          # -0 sum -> checksum +0
    assert oracle.hdr_verify(ff.ptr, 6) == (1, 200)


def test_null_chain_with_pseudo_header():
    ph = netcsum.HostBytes(bytes.fromhex("c0a80001c0a800c700060014"))
    v, err = oracle.data_calc(None, ph.ptr, 12)
    assert err == 200
    assert v == onp.hdr_calc(bytes.fromhex("c0a80001c0a800c700060014"))
    # odd pseudo-header with no buffers: the last octet is never summed (net_util.c:1601-1611)
    ph11 = netcsum.HostBytes(bytes.fromhex("c0a80001c0a800c7000600"))
    v11, _ = oracle.data_calc(None, ph11.ptr, 11)
    assert v11 == onp.hdr_calc(bytes.fromhex("c0a80001c0a800c70006"))
    assert onp.data_calc(None, bytes.fromhex("c0a80001c0a800c7000600"))[0] == v11


def test_invalid_protocol():
    ch = netcsum.Chain([{"data": b"abcd", "proto": netcsum.NET_PROTOCOL_TYPE_IGMP}])
    assert oracle.data_calc(ch.ptr, None, 0) == (0, 211)
    assert oracle.data_verify(ch.ptr, None, 0) == (0, 211)
    assert onp.data_calc([onp.Buf(b"abcd", proto=62)], None) == (0, 211)


def test_udp_pseudo_header_kat():
    """A UDP datagram whose checksum, computed with its pseudo-header and written back, verifies
    (the Tx->Rx round trip of net_udp.c:2891/2937 then :1934)."""
    ph = bytes.fromhex("0a000001" "0a000002" "00" "11" "000c")
    udp = bytearray(bytes.fromhex("d431" "0035" "000c" "0000" "61626364"))
    ch = netcsum.Chain([{"data": bytes(udp), "proto": netcsum.NET_PROTOCOL_TYPE_UDP_V4}])
    phb = netcsum.HostBytes(ph)
    v, err = oracle.data_calc(ch.ptr, phb.ptr, 12)
    assert err == 200
    udp[6:8] = v.to_bytes(2, "little")
    ch2 = netcsum.Chain([{"data": bytes(udp), "proto": netcsum.NET_PROTOCOL_TYPE_UDP_V4}])
    assert oracle.data_verify(ch2.ptr, phb.ptr, 12) == (1, 200)
    assert onp.data_verify([onp.Buf(bytes(udp), proto=70)], ph) == (1, 200)
