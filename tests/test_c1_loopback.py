"""Config C1 (BASELINE.json configs[0]): the IF/net_if_loopback.c UDP echo with 64-B datagrams.

The reference stack cannot run here (uC-CPU / uC-LIB / KAL are not vendored), so this test replays
the per-datagram checksum call sequence of SURVEY §3.1/§3.2 on real frame bytes:

  Tx  NetUDP_TxPktPrepareHdr  net_udp.c:2891  DataCalc(p_buf, &udp_pseudo_hdr, 12) (0 -> 0xFFFF, :2929)
      NetIPv4_TxPktPrepareHdr net_ipv4.c:9578 HdrCalc(ip_hdr, 20)
      NetIF_Loopback_Tx       net_if_loopback.c:731 copy into an Rx buffer
  Rx  NetIPv4_RxPktValidate   net_ipv4.c:5247 HdrVerify(ip_hdr, 20)
      NetUDP_RxPktValidate    net_udp.c:1934  DataVerify(p_buf, &udp_pseudo_hdr, 12)
  echo: swap addresses/ports and send back (udp_server.c:140/156 shape)

with NET_BUF fields set the way the stack sets them (ProtocolHdrType UDP_V4, TransportHdrIx =
IP header length, TransportHdrLen 8, DataLen 64). The CPU variant runs the oracle; the GPU variant
runs the product drop-in and must match the oracle value for value.
"""
import struct

import pytest

import netcsum
import oracle


def _ip_hdr(src, dst, total_len, ident):
    return bytearray(struct.pack("!BBHHHBBH4s4s", 0x45, 0, total_len, ident, 0x4000, 64, 17, 0, src, dst))


def _pseudo(src, dst, udp_len):
    return struct.pack("!4s4sBBH", src, dst, 0, 17, udp_len)


class Api:
    def __init__(self, gpu):
        self.gpu = gpu

    def data_calc(self, ch, ph):
        return netcsum.DataCalc(ch, ph.ptr, 12) if self.gpu else oracle.data_calc(ch, ph.ptr, 12)

    def data_verify(self, ch, ph):
        return netcsum.DataVerify(ch, ph.ptr, 12) if self.gpu else oracle.data_verify(ch, ph.ptr, 12)

    def hdr_calc(self, hb):
        return netcsum.HdrCalc(hb.ptr, 20) if self.gpu else oracle.hdr_calc(hb.ptr, 20)

    def hdr_verify(self, hb):
        return netcsum.HdrVerify(hb.ptr, 20) if self.gpu else oracle.hdr_verify(hb.ptr, 20)


def _tx(api, src, dst, sport, dport, payload, ident):
    udp_len = 8 + len(payload)
    ip = _ip_hdr(src, dst, 20 + udp_len, ident)
    udp = bytearray(struct.pack("!HHHH", sport, dport, udp_len, 0)) + payload
    frame = bytes(ip) + bytes(udp)
    ch = netcsum.Chain([{"data": frame, "proto": netcsum.NET_PROTOCOL_TYPE_UDP_V4, "transport_ix": 20,
                         "transport_hdr_len": 8, "data_len": len(payload)}])
    ph = netcsum.HostBytes(_pseudo(src, dst, udp_len))
    c, err = api.data_calc(ch.ptr, ph)
    assert err == netcsum.NET_UTIL_ERR_NONE
    if c == 0x0000:                                   # RFC 768: +0 is sent as -0 (net_udp.c:2929-2931)
        c = 0xFFFF
    udp[6:8] = c.to_bytes(2, "little")               # NET_UTIL_VAL_COPY_16 of the host-order value
    hb = netcsum.HostBytes(bytes(ip))
    h, err = api.hdr_calc(hb)
    assert err == netcsum.NET_UTIL_ERR_NONE
    ip[10:12] = h.to_bytes(2, "little")
    return bytes(ip) + bytes(udp), (c, h)


def _rx(api, frame):
    ip = frame[:20]
    src, dst = ip[12:16], ip[16:20]
    udp_len = struct.unpack("!H", frame[24:26])[0]
    hb = netcsum.HostBytes(ip)
    ok_ip, err = api.hdr_verify(hb)
    assert err == netcsum.NET_UTIL_ERR_NONE
    ch = netcsum.Chain([{"data": frame, "proto": netcsum.NET_PROTOCOL_TYPE_UDP_V4, "transport_ix": 20,
                         "transport_hdr_len": 8, "data_len": udp_len - 8}], offset=2)   # Rx buf offset
    ph = netcsum.HostBytes(_pseudo(src, dst, udp_len), 1)
    ok_udp, err = api.data_verify(ch.ptr, ph)
    assert err == netcsum.NET_UTIL_ERR_NONE
    return ok_ip, ok_udp


def _echo_session(api, n=64):
    src, dst = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    vals = []
    for i in range(n):
        payload = bytes((i * 7 + k * 13) & 0xFF for k in range(64))
        frame, cs = _tx(api, src, dst, 5000 + i, 7, payload, i)
        assert _rx(api, frame) == (1, 1)                      # loopback Rx validates
        reply, cs2 = _tx(api, dst, src, 7, 5000 + i, frame[28:], 0x8000 + i)   # echo back
        assert _rx(api, reply) == (1, 1)
        bad = bytearray(reply)
        bad[40] ^= 0x01                                       # corrupt payload: UDP fails, IP passes
        assert _rx(api, bytes(bad)) == (1, 0)
        bad = bytearray(reply)
        bad[8] ^= 0x01                                        # corrupt TTL: IP fails
        assert _rx(api, bytes(bad))[0] == 0
        vals.append((cs, cs2))
    return vals


def test_c1_loopback_echo_oracle():
    _echo_session(Api(gpu=False))


@pytest.mark.gpu
def test_c1_loopback_echo_gpu_dropin_matches_oracle():
    pytest.importorskip("torch")
    assert _echo_session(Api(gpu=True), 32) == _echo_session(Api(gpu=False), 32)
