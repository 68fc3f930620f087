"""GPU parity of ChkSumBatchVarLen on segments where the stack holds them: one TCP
segment per NET_BUF pool buffer at DataPtr + TransportHdrIx (/root/reference/Source/net_util.c:1627-1628,
1649; Source/net_tcp.c:1920), 1520-B and 2-KiB buffers, uniform 1480-B segments and the 20 / 556 / 1480-B
mix of 40 / 576 / 1500-B datagrams, against the oracle's NetUtil_16BitOnesCplChkSumDataCalc /
...DataVerify per segment (oracle/net_util_oracle.c).

The bytes between segments are random here, so a kernel that summed any of them would disagree with
the oracle. The batch's plan (varlen_runlen_kernel) sends segments with gaps in address order to the
live-sector stream (seg_live_varlen_kernel: only the 64-B sectors holding segment bytes are read)
from the second batch on the same descriptors; its runs out of order or past the 63-KiB reach take
16-lane groups. Other layouts stay in the stream kernel (packed runs streamed, others by 16-lane
groups). Reversed, shuffled, duplicated and far-apart descriptors, empty segments, odd offsets and odd
pseudo-header lengths are mixed in; every run length from 1 to 128."""
import zlib

import numpy as np
import pytest

import netcsum
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _defaults():
    yield
    netcsum.tune(netcsum.TUNE_TILE, -1)
    netcsum.tune(netcsum.TUNE_VARLEN_RUN_BYTES, -1)
    netcsum.tune(netcsum.TUNE_CHUNKS, 0)


def _pool(rng, n, slot, ix, mix, order):
    lens = (np.array([20, 556, 1480])[rng.choice(3, size=n, p=[7 / 12, 4 / 12, 1 / 12])] if mix
            else np.full(n, 1480)).astype(np.uint16)
    lens[rng.choice(n, size=n // 50, replace=False)] = 0                # empty segments
    odd = rng.random(n) < 0.1                                            # a few odd offsets (odd IP options)
    offs = (np.arange(n, dtype=np.uint64) * np.uint64(slot) + np.uint64(ix) + odd.astype(np.uint64))
    lens = np.minimum(lens, slot - ix - 1).astype(np.uint16)
    size = n * slot + 64
    if order == "far":                                                   # every 7th buffer 300 KiB further on
        offs = offs + (np.arange(n, dtype=np.uint64) // 7) * np.uint64(300 * 1024)
        size = int(offs[-1]) + slot + 64
    buf = rng.integers(0, 256, size=size, dtype=np.uint8)
    if order == "reversed":
        offs, lens = offs[::-1].copy(), lens[::-1].copy()
    elif order == "shuffled":
        perm = rng.permutation(n)
        offs, lens = offs[perm].copy(), lens[perm].copy()
    elif order == "duplicates":
        offs[1::9] = offs[0::9][: len(offs[1::9])]
        lens[1::9] = lens[0::9][: len(lens[1::9])]
    return buf, offs, lens


@pytest.mark.parametrize("order", ["sorted", "reversed", "shuffled", "duplicates", "far"])
@pytest.mark.parametrize("slot,ix,mix", [(1520, 34, False), (1520, 34, True), (2048, 84, False), (2048, 84, True)])
@pytest.mark.parametrize("plen", [0, 12, 11, 40])
def test_pool_segments_vs_oracle(order, slot, ix, mix, plen):
    key = zlib.crc32(f"{order}/{slot}/{mix}/{plen}".encode())
    rng = np.random.default_rng(key)
    n = 3000 + key % 10007      # (a batch size of its own: plans are keyed on the arrays' addresses and
                                # the count, and torch hands the next test the same addresses)
    buf, offs, lens = _pool(rng, n, slot, ix, mix, order)
    ph = rng.integers(0, 256, size=n * max(plen, 1), dtype=np.uint8) if plen else None
    b = torch.from_numpy(buf).to(DEV)
    o = torch.from_numpy(offs.view(np.int64)).to(DEV)
    ln = torch.from_numpy(lens.view(np.int16)).to(DEV)
    p = torch.from_numpy(ph).to(DEV) if plen else None
    want_c = oracle.batch_varlen(buf, offs, lens, ph, plen, plen, netcsum.OP_DATA_CALC)
    want_v = oracle.batch_varlen(buf, offs, lens, ph, plen, plen, netcsum.OP_DATA_VERIFY)
    launches = []
    for op_ in (netcsum.OP_DATA_CALC, netcsum.OP_DATA_VERIFY, netcsum.OP_DATA_CALC):
        want = want_c if op_ == netcsum.OP_DATA_CALC else want_v
        out = torch.zeros(n * (2 if op_ == netcsum.OP_DATA_CALC else 1), dtype=torch.uint8, device=DEV)
        netcsum.batch_varlen(b, o, ln, p, plen, plen, n, out, op_)
        torch.cuda.synchronize()
        launches.append(netcsum.last_launch())
        got = out.cpu().numpy().view(np.uint16) if op_ == netcsum.OP_DATA_CALC else out.cpu().numpy()
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (op_, launches[-1], [(int(i), int(got[i]), int(want[i]), int(offs[i]), int(lens[i]))
                                                   for i in bad[:6]])
    # the batch's plan (the sampler of the first call): segments with gaps in address order take the
    # live-sector stream from the second call on the same descriptors (1480-B segments: runs of 8 at
    # depth 4 in 1520-B buffers, 16 at depth 8 in 2-KiB ones; the mix: as long as the reach allows, 41 /
    # 30 at depth 4); its own sampler block keeps it
    for last in launches:
        assert last.split("<")[0] in ("seg_stream_varlen_kernel", "seg_live_varlen_kernel", "seg_pipe_kernel"), last
    if order == "sorted":
        for last in launches[1:]:
            run, depth = ((8, 4) if slot == 1520 else (16, 8)) if not mix else ((41 if slot == 1520 else 30), 4)
            assert "plan=pool(live)" in last and f"D={depth}" in last, last
            assert f"segs_per_wave={run}" in last, last


@pytest.mark.parametrize("spw", [1, 2, 7, 31, 64, 65, 128])
@pytest.mark.parametrize("depth", [4, 8])
@pytest.mark.parametrize("order", ["sorted", "duplicates"])
def test_pool_segments_every_run_length(spw, depth, order):
    """Fixed runs (TUNE_TILE) of 1..128 segments in 2-KiB buffers with the mix, 4 and 8 pieces in flight:
    the first call in the stream kernel (its 16-lane groups for runs with gaps), the second in the
    live-sector stream of the batch's plan at that run length (<= 64; past it the plan's) — with some
    descriptors listed twice, its runs that hold them take the 16-lane groups."""
    netcsum.tune(netcsum.TUNE_TILE, spw)
    netcsum.tune(netcsum.TUNE_CHUNKS, depth)
    rng = np.random.default_rng(spw * 10 + depth)
    n = 2000 + spw * 3 + depth + (7 if order == "duplicates" else 0)
    buf, offs, lens = _pool(rng, n, 2048, 84, True, order)
    ph = rng.integers(0, 256, size=n * 12, dtype=np.uint8)
    want = oracle.batch_varlen(buf, offs, lens, ph, 12, 12, netcsum.OP_DATA_CALC)
    args = (torch.from_numpy(buf).to(DEV), torch.from_numpy(offs.view(np.int64)).to(DEV),
            torch.from_numpy(lens.view(np.int16)).to(DEV), torch.from_numpy(ph).to(DEV))
    for call in range(2):
        out = torch.zeros(n, dtype=torch.int16, device=DEV)
        netcsum.batch_varlen(*args, 12, 12, n, out, netcsum.OP_DATA_CALC)
        torch.cuda.synchronize()
        last = netcsum.last_launch()
        assert np.array_equal(out.cpu().numpy().view(np.uint16), want), (call, last)
    if spw <= 64:
        assert "plan=pool(live)" in last and f"D={depth}" in last and f"segs_per_wave={spw}" in last, last
    else:                                                                # past the live form's runs
        assert last.startswith("seg_stream_varlen_kernel"), last


def test_pool_segments_full_size_properties():
    """1 M segments of the mix in 2-KiB buffers (the probe's layout): Calc, the checksums written into
    each segment's checksum field (TCP: +16), then Verify reads every segment OK; one corrupted byte
    inside a segment is caught, one between segments is not read; a 4096-segment oracle sample."""
    n, slot, ix = 1 << 20, 2048, 84
    rng = np.random.default_rng(9)
    lens = np.array([20, 556, 1480])[rng.choice(3, size=n, p=[7 / 12, 4 / 12, 1 / 12])].astype(np.uint16)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(slot) + np.uint64(ix)
    b = torch.randint(0, 256, (n * slot + 64,), dtype=torch.uint8, device=DEV)
    o = torch.from_numpy(offs.view(np.int64)).to(DEV)
    ln = torch.from_numpy(lens.view(np.int16)).to(DEV)
    ph = torch.randint(0, 256, (n * 12,), dtype=torch.uint8, device=DEV)
    bv = b[: n * slot].view(n, slot)
    bv[:, ix + 16:ix + 18] = 0                                           # the TCP checksum fields
    out = torch.zeros(n, dtype=torch.int16, device=DEV)
    netcsum.batch_varlen(b, o, ln, ph, 12, 12, n, out, netcsum.OP_DATA_CALC)
    torch.cuda.synchronize()
    smp = np.sort(rng.choice(n, size=4096, replace=False))
    hb = b.cpu().numpy()
    segs = np.concatenate([hb[int(offs[i]):int(offs[i]) + int(lens[i])] for i in smp])
    so = np.zeros(len(smp), np.uint64)
    so[1:] = np.cumsum(lens[smp][:-1].astype(np.uint64))
    phs = ph.cpu().numpy().reshape(n, 12)[smp].reshape(-1)
    assert np.array_equal(out.cpu().numpy().view(np.uint16)[smp],
                          oracle.batch_varlen(segs, so, lens[smp].copy(), phs, 12, 12, netcsum.OP_DATA_CALC))
    c = out.view(torch.uint8).view(n, 2)                                 # host-order u16 -> the field's bytes
    bv[:, ix + 16:ix + 18] = c
    ok = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.batch_varlen(b, o, ln, ph, 12, 12, n, ok, netcsum.OP_DATA_VERIFY)
    torch.cuda.synchronize()
    assert bool((ok == 1).all().item())
    k = int(np.nonzero(lens == 1480)[0][77])
    bv[k, ix + 1000] ^= 0x5A
    bv[k + 1, ix + int(lens[k + 1]) + 8] ^= 0xA5                        # past segment k + 1's end
    netcsum.batch_varlen(b, o, ln, ph, 12, 12, n, ok, netcsum.OP_DATA_VERIFY)
    torch.cuda.synchronize()
    f = ok.cpu().numpy()
    assert f[k] == 0 and (np.delete(f, k) == 1).all()
