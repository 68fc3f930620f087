"""Host threading of the drop-in on the GPU (the reference is reentrant — no statics in
net_util.c:159-449 — and serialised by the stack's global lock, Source/net.c:550; the GPU C ABI must
be safe from one host thread per device):

* the plain C caller (tests/c/dropin_caller.c, standalone build) with NETCSUM_EXPECT_GPU=1: every
  device call succeeds and matches its own RFC 1071 sum, incl. two pthreads on one device and
  chains of up to 1000 buffers;
* two Python threads on one device (ctypes drops the GIL during the call) against the oracle;
* one thread per device when the box has more than one GPU;
* per-thread contexts are released at thread exit and by NetUtil_MI355X_ThreadRelease: 48 threads
  that each stage a > 16 KiB packet leave no device memory behind.
"""
import os
import random
import subprocess
import threading

import pytest

import netcsum
import oracle
from helpers import rand_buf, rand_chain

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_caller_on_gpu():
    exe = os.path.join(REPO, "tests", "c", "build", "standalone")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "c"), "build/standalone"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, NETCSUM_EXPECT_GPU="1"))
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert r.stdout.startswith("ok ") and "device_missing=0" in r.stdout, r.stdout


def test_burst_caller_on_gpu():
    """tests/c/burst_caller.c with the GPU: a 4096-frame host ring through RxBurstHost (actions and
    counters equal the caller's own RFC 1071 verdicts) and TxBurstHost (every frame verifies)."""
    for exe_name in ("burst", "burst_instack"):
        exe = os.path.join(REPO, "tests", "c", "build", exe_name)
        if not os.path.exists(exe):
            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "c"), "build/" + exe_name], check=True)
        env = dict(os.environ, NETCSUM_EXPECT_GPU="1")
        r = subprocess.run([exe], capture_output=True, text=True, timeout=110, env=env)
        assert r.returncode == 0, r.stdout + r.stderr[-3000:]
        assert r.stdout.startswith("ok ") and "gpu=1" in r.stdout, r.stdout


def _cases(seed, n):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        ch = netcsum.Chain(rand_chain(rng, rng.choice([20, 72, 1480, rng.randint(0, 20000)]), rng.randint(1, 5)))
        ph = netcsum.HostBytes(bytes(rng.randrange(256) for _ in range(12)), rng.randint(0, 3))
        out.append((ch, ph, oracle.data_calc(ch.ptr, ph.ptr, 12), oracle.data_verify(ch.ptr, ph.ptr, 12)))
    return out


def _worker(cases, dev, errors):
    try:
        torch.cuda.set_device(dev)
        for k, (ch, ph, want_c, want_v) in enumerate(cases):
            got = netcsum.DataCalc(ch.ptr, ph.ptr, 12)
            if got != want_c:
                errors.append((dev, k, got, want_c))
            if netcsum.DataVerify(ch.ptr, ph.ptr, 12) != want_v:
                errors.append((dev, k, "verify"))
    except Exception as e:  # noqa: BLE001 — reported through the list
        errors.append(repr(e))
    finally:
        netcsum.thread_release()


def _run_threads(devs, per_thread=150):
    errors = []
    ths = [threading.Thread(target=_worker, args=(_cases(11 + i, per_thread), d, errors)) for i, d in enumerate(devs)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ths), "a drop-in thread did not finish"
    assert errors == []


def test_two_threads_one_device():
    _run_threads([0, 0])


def test_one_thread_per_device():
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("one GPU on this box")
    _run_threads(list(range(min(n, 8))), per_thread=60)


def test_thread_contexts_released():
    """Each thread stages a 1.2 MB reassembled datagram (20 x 60000-B buffers: a 1.2 MB device
    staging buffer, streams, pinned memory). After 48 such threads have exited (58 MB if leaked),
    device memory is back where it was: contexts do not leak."""
    rng = random.Random(3)
    ch = netcsum.Chain([rand_buf(rng, 60000) for _ in range(20)])
    want = oracle.data_calc(ch.ptr, None, 0)

    def one(errors):
        try:
            if netcsum.DataCalc(ch.ptr, None, 0) != want:
                errors.append("mismatch")
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    errors = []
    t = threading.Thread(target=one, args=(errors,))
    t.start()
    t.join()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(48):
        t = threading.Thread(target=one, args=(errors,))
        t.start()
        t.join(timeout=30)
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    assert errors == []
    assert free0 - free1 < 32 << 20, f"{(free0 - free1) >> 20} MiB of device memory not released"
    # explicit release on this thread, then the drop-in re-creates its context on the next call
    assert netcsum.thread_release() == 200
    assert netcsum.DataCalc(ch.ptr, None, 0) == want
    assert netcsum.thread_release() == 200


def test_scratch_buffers_many_threads_many_streams():
    """Every scratch lease is per thread and per stream (netcsum_abi.hip ScratchLease): 4 threads x 24
    streams each — more streams than a thread's 16 slots, so slots are evicted and re-created while
    launches on other streams are in flight — run at once, per stream:
      * two-pass Tx finalize (TUNE_TX_PASSES 2, per thread): the event-ordered 8-B records lease;
      * a two-pass chain batch: the event-ordered per-piece records lease;
      * an IPv6 lane-group Rx batch without a flags array (TUNE_KERNEL 2 around it): the event-ordered
        deferral word + flags lease, with datagrams whose extension chains the walk pass finishes;
      * an adaptive-run varlen batch: the unordered run-word lease.
    Every result equals the oracle's."""
    import struct

    import numpy as np
    import oracle_packets as op
    from chains import make_chain_batch
    from packets import ext_body, make_packet, make_packet_v6, packed_batch

    rng = random.Random(77)
    stride, n_pkt = 1500, 96
    tx_in = np.zeros(n_pkt * stride + 64, np.uint8)
    tx_want = tx_in.copy()
    for i in range(n_pkt):
        p = make_packet(rng, rng.choice(["tcp", "udp", "icmp"]), payload=rng.randint(100, 1300))[:stride]
        tx_in[i * stride:i * stride + len(p)] = np.frombuffer(p, np.uint8)
        q, _ = op.tx_finalize(bytes(tx_in[i * stride:(i + 1) * stride]))
        tx_want[i * stride:(i + 1) * stride] = np.frombuffer(q, np.uint8)
    segs = [rng.randbytes(rng.randint(40, 3000)) for _ in range(400)]
    vbuf, voff, vlen = packed_batch(segs, rng, trailer=False)
    vwant = oracle.batch_varlen(vbuf, voff, vlen, None, 0, 0)
    cb = make_chain_batch(rng, 64, max_pieces=12)
    cwant = cb.expect(0)
    v6 = []
    for i in range(128):                                  # every 4th behind a long Destination Options header
        inner = make_packet_v6(rng, rng.choice(["tcp", "udp", "icmp_echo"]), payload=rng.randint(24, 900))
        if i % 4 == 0:
            u = rng.randint(8, 30)
            body = struct.pack("!BB", inner[6], u - 1) + ext_body(rng, 60, u * 8 - 2) + inner[40:]
            inner = inner[:4] + struct.pack("!HB", len(body), 60) + inner[7:40] + body
        v6.append(inner)
    v6buf, v6off, v6len = packed_batch(v6, rng)
    v6want = np.array([op.rx_validate_v6(bytes(v6buf[o:o + n])) for o, n in zip(v6off.tolist(), v6len.tolist())], np.uint8)
    import oracle_offload as oo
    v6frames = [bytes(v6buf[o:o + n]) for o, n in zip(v6off.tolist(), v6len.tolist())]
    v6act = np.array([netcsum.rx_action(int(f), oo.transport_proto(fr), True) for f, fr in zip(v6want, v6frames)],
                     np.uint8)
    errors = []

    def worker(seed):
        try:
            torch.cuda.set_device(0)
            netcsum.tune(netcsum.TUNE_TX_PASSES, 2)       # per thread: Tx records even for 96 datagrams
            streams = [torch.cuda.Stream() for _ in range(24)]
            with torch.cuda.stream(streams[0]):
                vb = torch.from_numpy(vbuf).cuda()
                vo = torch.from_numpy(voff.astype(np.int64)).cuda()
                vl = torch.from_numpy(vlen.view(np.int16)).cuda()
                cbase = torch.from_numpy(cb.base).cuda()
                coff = torch.from_numpy(cb.piece_off.view(np.int64)).cuda()
                clen = torch.from_numpy(cb.piece_len.view(np.int16)).cuda()
                cfirst = torch.from_numpy(cb.chain_first.view(np.int32)).cuda()
                cph = torch.from_numpy(cb.pseudo).cuda()
                v6b = torch.from_numpy(v6buf).cuda()
                v6o = torch.from_numpy(v6off.view(np.int64)).cuda()
                v6l = torch.from_numpy(v6len.view(np.int16)).cuda()
            streams[0].synchronize()
            for rnd in range(3):
                res = []
                for s in streams:
                    with torch.cuda.stream(s):
                        b = torch.from_numpy(tx_in).cuda()
                        o = torch.empty(len(segs), dtype=torch.int16, device="cuda")
                        co = torch.empty(cb.n, dtype=torch.int16, device="cuda")
                        act = torch.full((len(v6),), 0xEE, dtype=torch.uint8, device="cuda")
                        netcsum.tx_finalize_ipv4(b, n_pkt, stride=stride, pkt_len=stride, stream=s)
                        netcsum.batch_chains(cbase, coff, clen, cfirst, cph, cb.pseudo_stride, cb.pseudo_len, cb.n,
                                             co, stream=s)
                        netcsum.tune(netcsum.TUNE_KERNEL, 2)
                        netcsum.rx_burst(v6b, len(v6), act, off=v6o, lens=v6l, stream=s)
                        netcsum.tune(netcsum.TUNE_KERNEL, 0)
                        netcsum.batch_varlen(vb, vo, vl, None, 0, 0, len(segs), o, stream=s)
                        res.append((b, o, co, act))
                for s, (b, o, co, act) in zip(streams, res):
                    s.synchronize()
                    if not np.array_equal(b.cpu().numpy(), tx_want):
                        errors.append((seed, rnd, "tx"))
                    if not np.array_equal(o.cpu().numpy().view(np.uint16), vwant):
                        errors.append((seed, rnd, "varlen"))
                    if not np.array_equal(co.cpu().numpy().view(np.uint16), cwant):
                        errors.append((seed, rnd, "chains"))
                    if not np.array_equal(act.cpu().numpy(), v6act):
                        errors.append((seed, rnd, "v6 lane-group rx"))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
        finally:
            netcsum.thread_release()

    ths = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=200)
    assert not any(t.is_alive() for t in ths)
    assert errors == []


def test_tuning_applies_to_the_calling_thread_only():
    """NetUtil_MI355X_Tune is per host thread: the main thread forcing the lane-group packet kernel
    (TUNE_KERNEL 2) and runs of 4 segments does not change another thread's launches, which take the
    default forms; results are the oracle's either way."""
    import numpy as np
    n, L = 4096, 1500
    rng = np.random.default_rng(5)
    seg = rng.integers(0, 256, size=n * L, dtype=np.uint8)
    want = oracle.batch_strided(seg, L, L, None, 0, 0, n, 0)
    d = torch.from_numpy(seg).cuda()
    out_main = torch.zeros(n, dtype=torch.int16, device="cuda")
    netcsum.tune(netcsum.TUNE_KERNEL, 2)
    try:
        netcsum.batch_strided(d, L, L, None, 0, 0, n, out_main)
        torch.cuda.synchronize()
        desc_main = netcsum.last_launch()
        seen = {}

        def other():
            torch.cuda.set_device(0)
            o = torch.zeros(n, dtype=torch.int16, device="cuda")
            netcsum.batch_strided(d, L, L, None, 0, 0, n, o)
            torch.cuda.synchronize()
            seen["desc"] = netcsum.last_launch()
            seen["ok"] = np.array_equal(o.cpu().numpy().view(np.uint16), want)
            netcsum.thread_release()

        t = threading.Thread(target=other)
        t.start()
        t.join(timeout=60)
    finally:
        netcsum.tune(netcsum.TUNE_KERNEL, 0)
    assert desc_main.startswith("seg_pipe_kernel"), desc_main
    assert seen["desc"].startswith("seg_stream_kernel"), seen
    assert seen["ok"] and np.array_equal(out_main.cpu().numpy().view(np.uint16), want)
