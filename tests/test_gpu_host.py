"""GPU parity of the host-memory forms (include/netcsum_mi355x.h (2e)): every
pointer in host memory, the batch pipelined in chunks over three streams (H2D of each chunk's byte
span and rebased descriptors -> the device form -> D2H of the results; Tx writes the span back).
Results equal the oracle's for 1, 2, 3, 7 and 64 chunks, packed and unsorted offset/length batches,
strided batches, odd base offsets; an overlapping Tx batch (chunk spans that overlap) is still exact."""
import os
import random

import numpy as np
import pytest

import netcsum
import oracle
import oracle_offload as oo
import oracle_packets as op
from packets import KINDS, KINDS6, make_packet, make_packet_v6, packed_batch

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _defaults():
    yield
    netcsum.tune(netcsum.TUNE_KERNEL, 0)
    netcsum.tune(netcsum.TUNE_TX_PASSES, 0)


def _pinned(a):
    t = torch.from_numpy(np.ascontiguousarray(a)).pin_memory()
    return t


@pytest.mark.parametrize("chunks", [1, 3, 7, 64])
@pytest.mark.parametrize("op_", [netcsum.OP_DATA_CALC, netcsum.OP_DATA_VERIFY])
def test_varlen_host_vs_oracle(chunks, op_):
    rng = np.random.default_rng(chunks * 3 + op_)
    n = 3000
    lens = rng.integers(40, 9001, size=n).astype(np.uint16)
    lens[::101] = rng.integers(0, 40, size=len(lens[::101]))
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    off += 5
    data = rng.integers(0, 256, size=int(off[-1]) + int(lens[-1]) + 64, dtype=np.uint8)
    ph = rng.integers(0, 256, size=n * 12, dtype=np.uint8)
    want = oracle.batch_varlen(data, off, lens, ph, 12, 12, op_)
    hb, ho, hl, hp = _pinned(data), _pinned(off.view(np.int64)), _pinned(lens.view(np.int16)), _pinned(ph)
    out = torch.zeros(n * (2 if op_ == netcsum.OP_DATA_CALC else 1), dtype=torch.uint8).pin_memory()
    netcsum.batch_varlen_host(hb, ho, hl, hp, 12, 12, n, out, op_, n_chunks=chunks)
    got = out.numpy().view(np.uint16) if op_ == netcsum.OP_DATA_CALC else out.numpy()
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]


def test_varlen_host_unsorted_and_pageable():
    """Reversed and interleaved offsets (chunk spans overlap: each chunk copies its own span) from
    pageable numpy memory, no pseudo-header, HdrCalc."""
    rng = np.random.default_rng(2)
    n = 1200
    lens = rng.integers(1, 1600, size=n).astype(np.uint16)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    perm = rng.permutation(n)
    off, lens = off[perm].copy(), lens[perm].copy()
    data = rng.integers(0, 256, size=int((off + lens).max()) + 64, dtype=np.uint8)
    out = np.zeros(n, np.uint16)
    netcsum.batch_varlen_host(data, off, lens, None, 0, 0, n, out, netcsum.OP_HDR_CALC, n_chunks=5)
    assert np.array_equal(out, oracle.batch_varlen(data, off, lens, None, 0, 0, netcsum.OP_HDR_CALC))


def _mixed(rng, n, max_payload):
    out = []
    for _ in range(n):
        if rng.random() < 0.5:
            out.append(make_packet(rng, rng.choice(KINDS), payload=rng.randint(0, max_payload)))
        else:
            out.append(make_packet_v6(rng, rng.choice(KINDS6), payload=rng.randint(0, max_payload)))
    return out


@pytest.mark.parametrize("chunks", [1, 2, 7])
def test_rx_and_burst_host_varlen(chunks):
    rng = random.Random(30 + chunks)
    pkts = _mixed(rng, 1500, 1400)
    buf, offs, lens = packed_batch(pkts, rng)
    frames = [bytes(buf[o:o + n]) for o, n in zip(offs.tolist(), lens.tolist())]
    want_f = np.array([op.rx_validate_ip(f) for f in frames], np.uint8)
    want_a = np.array([netcsum.rx_action(int(x), oo.transport_proto(f), len(f) and f[0] >> 4 == 6)
                       for x, f in zip(want_f, frames)], np.uint8)
    hb = _pinned(buf)
    fl = np.zeros(len(pkts), np.uint8)
    netcsum.rx_validate_ip_host(hb, len(pkts), fl, off=offs, lens=lens, n_chunks=chunks)
    assert np.array_equal(fl, want_f)
    act = np.full(len(pkts), 0xEE, np.uint8)
    fl2 = np.zeros(len(pkts), np.uint8)
    netcsum.rx_burst_host(hb, len(pkts), act, flags=fl2, off=offs, lens=lens, n_chunks=chunks)
    assert np.array_equal(act, want_a) and np.array_equal(fl2, want_f)
    assert np.array_equal(hb.numpy(), buf)                       # Rx never writes the frames


@pytest.mark.parametrize("chunks", [1, 3, 64])
def test_tx_host_strided(chunks):
    rng = random.Random(40 + chunks)
    n, stride = 2000, 1536
    pkts = _mixed(rng, n, 1300)
    buf = np.frombuffer(rng.randbytes(n * stride + 64), np.uint8).copy()
    for i, p in enumerate(pkts):
        p = p[:stride]
        buf[i * stride:i * stride + len(p)] = np.frombuffer(p, np.uint8)
    want = buf.copy()
    want_f = np.zeros(n, np.uint8)
    for i in range(n):
        q, want_f[i] = op.tx_finalize_ip(bytes(buf[i * stride:(i + 1) * stride]), True)
        want[i * stride:(i + 1) * stride] = np.frombuffer(q, np.uint8)
    hb = _pinned(buf)
    fl = np.zeros(n, np.uint8)
    netcsum.tx_finalize_ip_host(hb, n, fl, stride=stride, pkt_len=stride, n_chunks=chunks)
    assert np.array_equal(hb.numpy(), want) and np.array_equal(fl, want_f)


def test_tx_burst_host_varlen_and_overlap():
    rng = random.Random(50)
    pairs = []
    for i in range(1200):
        pkt = (make_packet if i % 2 else make_packet_v6)(rng, rng.choice(["tcp", "udp", "udp"]),
                                                         payload=rng.randint(0, 1200))
        csum = rng.random() < 0.8
        pairs.append((oo.tx_stack_offload(pkt, csum), op.tx_finalize_ip(pkt, csum)[0]))
    buf, offs, lens = packed_batch([f for f, _ in pairs], rng, trailer=False)
    want = buf.copy()
    for (_, r), o in zip(pairs, offs.tolist()):
        want[o:o + len(r)] = np.frombuffer(r, np.uint8)
    hb = _pinned(buf)
    netcsum.tx_burst_host(hb, len(pairs), off=offs, lens=lens, n_chunks=6)
    assert np.array_equal(hb.numpy(), want)
    # the same frames listed evens first, then odds: the chunks' spans overlap (each chunk's records
    # patch only its own datagrams' fields), same bytes
    perm = np.concatenate([np.arange(0, len(pairs), 2), np.arange(1, len(pairs), 2)])
    hb2 = _pinned(buf)
    netcsum.tx_burst_host(hb2, len(pairs), off=offs[perm].copy(), lens=lens[perm].copy(), n_chunks=6)
    assert np.array_equal(hb2.numpy(), want)


@pytest.mark.parametrize("kernel,passes", [(0, 2), (0, 1), (2, 0)])
@pytest.mark.parametrize("chunks", [1, 5, 64])
def test_tx_host_records_every_kernel_form(kernel, passes, chunks):
    """Which fields a datagram had written comes from whichever Tx kernel wrote them: the run-stream
    kernel (two passes: the scatter pass; one pass: its epilogue), the lane-group kernel
    (TUNE_KERNEL 2), and the IPv6 walk pass for chains past the first kernel's window; UDP datagrams
    without a checksum get their 0 written; malformed ones nothing. Pageable numpy memory, odd lead."""
    import struct
    from packets import ext_body
    netcsum.tune(netcsum.TUNE_KERNEL, kernel)
    netcsum.tune(netcsum.TUNE_TX_PASSES, passes)
    rng = random.Random(700 + 10 * kernel + passes + chunks)
    n, stride, lead = 900, 1100, 3
    pkts = []
    for i in range(n):
        if i % 3 == 0:                                   # IPv6 with a long Destination Options header
            inner = make_packet_v6(rng, rng.choice(["tcp", "udp", "icmp_echo"]), payload=rng.randint(24, 600))
            u = rng.randint(1, 30)
            body = struct.pack("!BB", inner[6], u - 1) + ext_body(rng, 60, u * 8 - 2) + inner[40:]
            pkts.append(inner[:4] + struct.pack("!HB", len(body), 60) + inner[7:40] + body)
        elif i % 3 == 1:
            pkts.append(make_packet(rng, rng.choice(KINDS), payload=rng.randint(0, 1000)))
        else:
            pkts.append(make_packet_v6(rng, rng.choice(KINDS6), payload=rng.randint(0, 1000)))
    buf = np.frombuffer(rng.randbytes(lead + n * stride + 64), np.uint8).copy()
    for i, p in enumerate(pkts):
        p = p[:stride]
        buf[lead + i * stride:lead + i * stride + len(p)] = np.frombuffer(p, np.uint8)
    want = buf.copy()
    want_f = np.zeros(n, np.uint8)
    for i in range(n):
        o = lead + i * stride
        q, want_f[i] = op.tx_finalize_ip(bytes(buf[o:o + stride]), True)
        want[o:o + stride] = np.frombuffer(q, np.uint8)
    got = buf.copy()
    fl = np.zeros(n, np.uint8)
    netcsum.tx_finalize_ip_host(got[lead:], n, fl, stride=stride, pkt_len=stride, n_chunks=chunks)
    assert netcsum.last_launch().startswith("pkt_batch_kernel" if kernel == 2 else "pkt_stream_kernel")
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(j), (int(j) - lead) // stride, (int(j) - lead) % stride) for j in bad[:8]]
    assert np.array_equal(fl, want_f)
    assert (want_f & op.L4_CHECKED).any() and (want_f & op.MALFORMED).any()


@pytest.mark.parametrize("n", [1, 2, 17, 64, 256, 4096, 4097])
@pytest.mark.parametrize("form", ["strided", "offlen", "sparse"])
def test_rx_burst_host_zero_copy(n, form):
    """NIC-burst sizes with n_chunks 0 from a pinned ring: the kernel reads the ring in place and the
    host polls a completion word (rx_burst_zero_copy, up to 4096 frames; 4097 takes the copy path) or
    the results themselves (TUNE_BURST_ZERO_COPY 2), or the resident burst server takes the burst
    from a posted line (3); the same results as the copy pipeline (TUNE_BURST_ZERO_COPY 0), a pageable
    ring (copy path) and the oracle, for RxBurstHost and RxValidateIPHost; the ring is never written.
    Forms: 1520-B slots at +14 (strided: the whole-span stream; offlen: per-frame descriptors) and
    2048-B slots at +64 with 1984 B present (sparse: the live-piece stream)."""
    rng = random.Random(900 + n + (form == "offlen") + 2 * (form == "sparse"))
    stride, lead = (2048, 64) if form == "sparse" else (1520, 14)
    pkts = [p[:stride - lead] for p in _mixed(rng, n, 1400)]
    buf = np.frombuffer(rng.randbytes(n * stride + 64), np.uint8).copy()
    for i, p in enumerate(pkts):
        buf[i * stride + lead:i * stride + lead + len(p)] = np.frombuffer(p, np.uint8)
    if form != "offlen":
        frames = [bytes(buf[i * stride + lead:(i + 1) * stride]) for i in range(n)]
        kw = {"stride": stride, "pkt_len": stride - lead}
        base = lambda b: b[lead:]                                   # noqa: E731
    else:
        offs = np.arange(n, dtype=np.uint64) * stride + 14
        lens = np.array([max(len(p), 46) for p in pkts], np.uint16)
        frames = [bytes(buf[o:o + m]) for o, m in zip(offs.tolist(), lens.tolist())]
        kw = {"off": offs, "lens": lens}
        base = lambda b: b                                          # noqa: E731
    want_f = np.array([op.rx_validate_ip(f) for f in frames], np.uint8)
    want_a = np.array([netcsum.rx_action(int(x), oo.transport_proto(f), len(f) and f[0] >> 4 == 6)
                       for x, f in zip(want_f, frames)], np.uint8)
    for zc, ring in ((1, _pinned(buf)), (2, _pinned(buf)), (3, _pinned(buf)), (0, _pinned(buf)), (3, buf.copy())):
        netcsum.tune(netcsum.TUNE_BURST_ZERO_COPY, zc)
        try:
            act = np.full(n, 0xEE, np.uint8)
            fl = np.zeros(n, np.uint8)
            netcsum.rx_burst_host(base(ring), n, act, flags=fl, **kw)
            assert np.array_equal(act, want_a) and np.array_equal(fl, want_f), (zc, type(ring))
            fl2 = np.zeros(n, np.uint8)
            netcsum.rx_validate_ip_host(base(ring), n, fl2, **kw)
            assert np.array_equal(fl2, want_f)
            act2 = np.full(n, 0xEE, np.uint8)
            netcsum.rx_burst_host(base(ring), n, act2, **kw)           # actions only
            assert np.array_equal(act2, want_a)
        finally:
            netcsum.tune(netcsum.TUNE_BURST_ZERO_COPY, 3)
        r = ring.numpy() if hasattr(ring, "numpy") else ring
        assert np.array_equal(r, buf)


@pytest.mark.parametrize("zc", [1, 2, 3])
def test_rx_burst_host_zero_copy_many_calls_and_threads(zc):
    """Back-to-back zero-copy bursts reuse one completion word per thread (tags never repeat a stale
    value), from two threads at once, each with its own ring (and, in mode 3, its own burst server)."""
    import threading
    errs = []

    def worker(seed):
        try:
            netcsum.tune(netcsum.TUNE_BURST_ZERO_COPY, zc)              # (per thread)
            rng = random.Random(seed)
            n, stride = 48, 1520
            for it in range(60):
                pkts = [p[:stride] for p in _mixed(rng, n, 1400)]
                buf = np.frombuffer(rng.randbytes(n * stride), np.uint8).copy()
                for i, p in enumerate(pkts):
                    buf[i * stride:i * stride + len(p)] = np.frombuffer(p, np.uint8)
                want = np.array([op.rx_validate_ip(bytes(buf[i * stride:(i + 1) * stride])) for i in range(n)], np.uint8)
                fl = np.zeros(n, np.uint8)
                netcsum.rx_validate_ip_host(_pinned(buf), n, fl, stride=stride, pkt_len=stride)
                if not np.array_equal(fl, want):
                    errs.append((seed, it))
            netcsum.thread_release()
        except Exception as e:                                        # noqa: BLE001
            errs.append(repr(e))
    th = [threading.Thread(target=worker, args=(s,)) for s in (1, 2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs


@pytest.mark.parametrize("n", [1, 3, 64, 500, 4096])
@pytest.mark.parametrize("form", ["strided", "offlen", "sparse"])
def test_tx_burst_host_zero_copy(n, form):
    """TxBurstHost with n_chunks 0 on a pinned ring (the IPv4 header at +14 of 1520-B slots, strided or
    per-frame offset/length; sparse: +64 of 2048-B slots): the checksum pass reads the ring in place
    and returns 8-B records that the host applies (tx_burst_zero_copy); IPv6 datagrams behind a long
    Destination Options header (flag EXT_HDR) are finished by the copy path. Same bytes and flags as
    the oracle and as the copy pipeline, and the zero-copy path (the server in mode 3) is the one
    taken in every layout (round-4 advisor: offset/length and sparse Tx took the copy path)."""
    import struct
    from packets import ext_body
    rng = random.Random(1300 + n + 7 * (form == "sparse"))
    stride, lead = (2048, 64) if form == "sparse" else (1520, 14)
    pairs = []
    for i in range(n):
        if i % 7 == 3:
            inner = make_packet_v6(rng, rng.choice(["tcp", "udp"]), payload=rng.randint(24, 900))
            u = rng.randint(10, 30)
            body = struct.pack("!BB", inner[6], u - 1) + ext_body(rng, 60, u * 8 - 2) + inner[40:]
            pkt = inner[:4] + struct.pack("!HB", len(body), 60) + inner[7:40] + body
        else:
            pkt = (make_packet(rng, rng.choice(["tcp", "udp", "udp", "icmp"]), payload=rng.randint(0, 1400)) if i % 2
                   else make_packet_v6(rng, rng.choice(["tcp", "udp", "udp", "icmp_echo"]), payload=rng.randint(0, 1400)))
        pkt = pkt[:stride - lead]
        csum = rng.random() < 0.8
        pairs.append((oo.tx_stack_offload(pkt, csum), op.tx_finalize_ip(pkt, csum)))
    buf = np.frombuffer(rng.randbytes(n * stride + 64), np.uint8).copy()
    want = buf.copy()
    want_f = np.zeros(n, np.uint8)
    for i, (f, (r, fl)) in enumerate(pairs):
        o = i * stride + lead
        buf[o:o + len(f)] = np.frombuffer(f, np.uint8)
        want[o:o + len(r)] = np.frombuffer(r, np.uint8)
    for i in range(n):                                     # the flags the oracle gives the stack's frame
        o = i * stride + lead
        want_f[i] = op.tx_finalize_ip(bytes(buf[o:(i + 1) * stride]), True)[1]
    for zc in (1, 2, 3, 0):
        netcsum.tune(netcsum.TUNE_BURST_ZERO_COPY, zc)
        try:
            hb = _pinned(buf)
            fl = np.zeros(n, np.uint8)
            if form != "offlen":
                netcsum.tx_burst_host(hb[lead:], n, fl, stride=stride, pkt_len=stride - lead)
            else:                                          # per-frame lengths (whole present bytes)
                offs = np.arange(n, dtype=np.uint64) * stride + lead
                lens = np.full(n, stride - lead, np.uint16)
                netcsum.tx_burst_host(hb, n, fl, off=offs, lens=lens)
            path = netcsum.last_launch()
        finally:
            netcsum.tune(netcsum.TUNE_BURST_ZERO_COPY, 3)
        if zc == 3:
            assert path.startswith("burst_server_kernel tx"), (zc, path)
        elif zc in (1, 2):
            assert "zero-copy" in path, (zc, path)
        else:
            assert "zero-copy" not in path, (zc, path)
        got = hb.numpy()
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (zc, [(int(j) // stride, int(j) % stride) for j in bad[:8]])
        # flags: the verdict bits of the finalize (UDP placeholder rules aside) on every datagram
        assert ((fl & op.MALFORMED) == (want_f & op.MALFORMED)).all()


def test_burst_server_idle_stop_and_relaunch():
    """The resident burst server (TUNE_BURST_ZERO_COPY 3) with a 20-us idle limit, bursts posted after
    pauses of 0..300 us: the server stops between many of them and bursts arrive while its blocks are
    closing (the post / closed-mark handshake, relaunch when a burst went unserved); every burst's
    results match the oracle; alternating Rx and Tx, strided and offset/length; a device-wide
    synchronisation returns once the server is idle."""
    import time
    rng = random.Random(77)
    stride, lead, n = 1520, 14, 40
    pkts = [p[:stride - lead] for p in _mixed(rng, n, 1400)]
    buf = np.frombuffer(rng.randbytes(n * stride), np.uint8).copy()
    for i, p in enumerate(pkts):
        buf[i * stride + lead:i * stride + lead + len(p)] = np.frombuffer(p, np.uint8)
    hb = _pinned(buf)
    want = np.array([op.rx_validate_ip(bytes(buf[i * stride + lead:(i + 1) * stride])) for i in range(n)], np.uint8)
    offs = np.arange(n, dtype=np.uint64) * stride + lead
    lens = np.full(n, stride - lead, np.uint16)
    tx_ref = _pinned(buf)                                           # Tx through the copy pipeline
    netcsum.tune(netcsum.TUNE_BURST_ZERO_COPY, 0)
    netcsum.tx_burst_host(tx_ref[lead:], n, None, stride=stride, pkt_len=stride - lead)
    tx_ref = tx_ref.numpy().copy()
    tb = _pinned(buf)
    netcsum.tune(netcsum.TUNE_BURST_ZERO_COPY, 3)
    netcsum.tune(netcsum.TUNE_BURST_SERVER_IDLE_US, 20)
    try:
        for it in range(400):
            k = rng.randint(1, n)
            fl = np.zeros(k, np.uint8)
            if it % 2:
                netcsum.rx_validate_ip_host(hb[lead:], k, fl, stride=stride, pkt_len=stride - lead)
            else:
                netcsum.rx_validate_ip_host(hb, k, fl, off=offs[:k], lens=lens[:k])
            assert np.array_equal(fl, want[:k]), it
            if it % 25 == 7:                                        # Tx of the first k slots of a copy
                tb.copy_(torch.from_numpy(buf))
                netcsum.tx_burst_host(tb[lead:], k, None, stride=stride, pkt_len=stride - lead)
                exp = buf.copy()
                exp[:k * stride] = tx_ref[:k * stride]
                assert np.array_equal(tb.numpy(), exp), it
            pause = rng.choice([0, 0, 5e-6, 2e-5, 5e-5, 3e-4])
            if pause:
                t = time.perf_counter() + pause
                while time.perf_counter() < t:
                    pass
        torch.cuda.synchronize()
    finally:
        netcsum.tune(netcsum.TUNE_BURST_SERVER_IDLE_US, 500)
        netcsum.tune(netcsum.TUNE_BURST_ZERO_COPY, 3)


@pytest.mark.parametrize("zc", [2, 3])
def test_zero_copy_ring_rewritten_between_bursts(zc):
    """The host rewrites its pinned ring in place between bursts (new frames in the same slots, as a
    NIC does): every burst sees the new bytes — a launch per burst through the launch's cache
    invalidation, the resident server (3) through its system-scope loads. Two ring contents
    alternate in one buffer, bursts of 1-8 frames back to back, Rx flags and Tx bytes checked each
    time against the oracle's for the content just written."""
    rng = random.Random(31 + zc)
    stride, lead, n = 1520, 14, 8
    rings, wants, txs = [], [], []
    for _ in range(2):
        pkts = [p[:stride - lead] for p in _mixed(rng, n, 1400)]
        b = np.frombuffer(rng.randbytes(n * stride), np.uint8).copy()
        for i, p in enumerate(pkts):
            b[i * stride + lead:i * stride + lead + len(p)] = np.frombuffer(p, np.uint8)
        rings.append(b)
        wants.append(np.array([op.rx_validate_ip(bytes(b[i * stride + lead:(i + 1) * stride])) for i in range(n)], np.uint8))
        t = _pinned(b)
        netcsum.tune(netcsum.TUNE_BURST_ZERO_COPY, 0)
        netcsum.tx_burst_host(t[lead:], n, None, stride=stride, pkt_len=stride - lead)
        txs.append(t.numpy().copy())
    hb = _pinned(rings[0])
    hv = hb.numpy()
    netcsum.tune(netcsum.TUNE_BURST_ZERO_COPY, zc)
    try:
        for it in range(300):
            j = it & 1
            k = rng.randint(1, n)
            hv[:] = rings[j]                                        # the host writes the ring in place
            fl = np.zeros(k, np.uint8)
            netcsum.rx_validate_ip_host(hb[lead:], k, fl, stride=stride, pkt_len=stride - lead)
            assert np.array_equal(fl, wants[j][:k]), (it, j, k)
            if it % 3 == 0:
                netcsum.tx_burst_host(hb[lead:], n, None, stride=stride, pkt_len=stride - lead)
                assert np.array_equal(hv, txs[j]), (it, j)
    finally:
        netcsum.tune(netcsum.TUNE_BURST_ZERO_COPY, 3)


def test_burst_server_process_exit_and_thread_release():
    """A process whose threads leave resident burst servers running exits cleanly: a child process
    posts bursts from its main thread and from a worker thread that ends without ThreadRelease (its
    context is released at thread exit, which stops its server), then exits while the main thread's
    server is still resident (stopped by the thread-local destructor at exit). Exit status 0, well
    inside the time limit; ThreadRelease on a live server returns at once."""
    import subprocess
    import sys
    import time
    code = r"""
import threading, time, numpy as np, torch, netcsum
stride, n = 1520, 32
buf = torch.zeros(n * stride, dtype=torch.uint8).pin_memory()
fl = np.zeros(n, np.uint8)
netcsum.rx_validate_ip_host(buf, n, fl, stride=stride, pkt_len=stride)
def worker():
    f2 = np.zeros(n, np.uint8)
    for _ in range(50):
        netcsum.rx_validate_ip_host(buf, n, f2, stride=stride, pkt_len=stride)
t = threading.Thread(target=worker); t.start(); t.join()
t0 = time.perf_counter(); netcsum.thread_release(); dt = time.perf_counter() - t0
assert dt < 0.5, dt
netcsum.rx_validate_ip_host(buf, n, fl, stride=stride, pkt_len=stride)   # a new server, left running
print("ok", flush=True)
"""
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(REPO, "uc-tcp-ip_amd"), env.get("PYTHONPATH", "")])
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stdout[-400:], r.stderr[-800:])
    assert time.perf_counter() - t0 < 100
