"""GPU parity of the header run-stream kernel (kernel 8, netcsum_hdrstream.hip: packed 16 / 20-B
headers, C3's shape) against the oracle (the C restatement of net_util.c:159-284): every base
offset in a 16-B line, batches from 1 header to several runs with partial last runs, run lengths
from 1 header to 4096, both load policies and pipeline depths, Calc and Verify ops, all-zero and
all-0xFF data (the 0 / 0xFFFF distinction), and the write-back property at 1 M headers."""
import numpy as np
import pytest

import netcsum
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _tuning():
    def reset():
        netcsum.tune(netcsum.TUNE_KERNEL, 0)
        netcsum.tune(netcsum.TUNE_CHUNKS, 0)
        netcsum.tune(netcsum.TUNE_TILE, -1)
        netcsum.tune(netcsum.TUNE_NT_LOADS, -1)
        netcsum.tune(netcsum.TUNE_STREAM_XCD, -1)
        netcsum.tune(netcsum.TUNE_STREAM_TOUCH, -1)
        netcsum.tune(netcsum.TUNE_HDR_BURST, -1)
    reset()
    yield
    reset()


def _run(host, lead, L, n, op):
    dev = torch.from_numpy(host).to(DEV)
    out = torch.zeros(n, dtype=torch.int16 if op in (0, 2) else torch.uint8, device=DEV)
    netcsum.batch_strided(dev[lead:], L, L, None, 0, 0, n, out, op)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    return got.view(np.uint16) if op in (0, 2) else got


@pytest.mark.parametrize("L", [20, 16])
@pytest.mark.parametrize("spw,depth,nt,xcd,touch", [(1024, 4, 1, -1, -1), (1, 4, 1, 1, 0), (7, 8, 0, -1, 1),
                                                    (64, 8, 1, 1, -1), (4096, 4, 0, 0, 0), (192, 4, 1, 1, 1),
                                                    (16, 4, 1, 0, 1), (384, 8, 1, -1, 1)])
@pytest.mark.parametrize("burst", [0, 1])      # results per run through LDS (spw <= 384, multiple of 16) or per piece
def test_hdrstream_vs_oracle(L, spw, depth, nt, xcd, touch, burst):
    netcsum.tune(netcsum.TUNE_KERNEL, 8)
    netcsum.tune(netcsum.TUNE_HDR_BURST, burst)
    netcsum.tune(netcsum.TUNE_STREAM_XCD, xcd)                   # launch options: block order, row touch
    netcsum.tune(netcsum.TUNE_STREAM_TOUCH, touch)
    netcsum.tune(netcsum.TUNE_TILE, spw)
    netcsum.tune(netcsum.TUNE_CHUNKS, depth)
    netcsum.tune(netcsum.TUNE_NT_LOADS, nt)
    rng = np.random.default_rng(L * 1000 + spw)
    for n in (1, 2, 51, 52, 257, spw, spw + 1, 3 * spw + 5, 20000):
        for lead in (0, 4, 8, 12):
            for pattern in ("random", "zero", "ff"):
                if pattern != "random" and n > 300:
                    continue
                size = lead + n * L + 64
                host = (rng.integers(0, 256, size=size, dtype=np.uint8) if pattern == "random" else
                        np.full(size, 0 if pattern == "zero" else 0xFF, np.uint8))
                for op in (2, 3):
                    got = _run(host, lead, L, n, op)
                    assert netcsum.last_launch().startswith(f"seg_hdrstream_kernel<M={L // 4},D={depth}")
                    want = oracle.batch_strided(host, L, L, None, 0, 0, n, op, seg_offset=lead)
                    bad = np.nonzero(got != want)[0]
                    assert bad.size == 0, (n, lead, pattern, op, bad[:5].tolist())


def test_hdrstream_round_trip_1M():
    netcsum.tune(netcsum.TUNE_KERNEL, 8)
    n, L = 1 << 20, 20
    hdr = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    netcsum.fill(hdr, n * L, 0x5EED0003, 0)
    h2 = hdr.view(n, L)
    h2[:, 10:12] = 0
    cs = torch.zeros(n, dtype=torch.int16, device=DEV)
    netcsum.batch_strided(hdr, L, L, None, 0, 0, n, cs, 2)
    torch.cuda.synchronize()
    assert netcsum.last_launch().startswith("seg_hdrstream_kernel"), netcsum.last_launch()
    h2[:, 10:12] = cs.view(torch.uint8).view(n, 2)
    ok = torch.zeros(n, dtype=torch.uint8, device=DEV)
    netcsum.batch_strided(hdr, L, L, None, 0, 0, n, ok, 3)
    torch.cuda.synchronize()
    assert bool(ok.all())
