"""The C restatement's per-datagram packet sequence (oracle Oracle_PktBatch: the CPU line of the
fused packet rows in tools/bench_configs.py) against the packet oracle (oracle/oracle_packets.py):
well-formed IPv4 (IP options included) and IPv6 TCP / UDP datagrams, Tx bytes equal, Rx verdict bits
equal on the finalized and on corrupted datagrams."""
import random

import numpy as np

import oracle
import oracle_packets as op
from packets import make_packet, make_packet_v6


def _batch(rng, n, stride):
    buf = np.zeros(n * stride, np.uint8)
    for i in range(n):
        kind = rng.choice(["tcp", "udp"])
        p = (make_packet if i % 2 else make_packet_v6)(rng, kind, payload=rng.randint(0, stride - 120))
        p = bytearray(p)
        if i % 2:
            p[10:12] = b"\x12\x34"                                   # stale IPv4 header checksum
        buf[i * stride:i * stride + len(p)] = np.frombuffer(bytes(p), np.uint8)
    return buf


def test_pkt_batch_tx_and_rx_equal_packet_oracle():
    rng = random.Random(5)
    n, stride = 400, 1600
    buf = _batch(rng, n, stride)
    want = buf.copy()
    for i in range(n):
        q, _ = op.tx_finalize_ip(bytes(buf[i * stride:(i + 1) * stride]), True)
        want[i * stride:(i + 1) * stride] = np.frombuffer(q, np.uint8)
    got = buf.copy()
    f_tx = oracle.pkt_batch(got, stride, stride, n, True, n_threads=2)
    assert np.array_equal(got, want)
    assert (f_tx == 7).all()
    f_rx = oracle.pkt_batch(got, stride, stride, n, False, n_threads=2)
    assert (f_rx == 7).all()
    bad = got.copy()
    for i in range(0, n, 7):
        bad[i * stride + 30 + rng.randrange(40)] ^= 0x01
    f_bad = oracle.pkt_batch(bad, stride, stride, n, False)
    want_bad = np.array([op.rx_validate_ip(bytes(bad[i * stride:(i + 1) * stride])) & 7 for i in range(n)], np.uint8)
    assert np.array_equal(f_bad, want_bad)
    assert (f_bad != 7).sum() >= n // 7 - 1
