"""The hand-counted vmcnt waits of seg_hdr_kernel<P,S,H> (netcsum_hdr.hip), turned into a test.

Every reachable instance runs with a grid of ONE block (4 waves, tiles dealt round-robin) and
n = 4 * cnt * 64H headers, so every wave owns exactly cnt tiles, for cnt = 1 .. S+1: each wave then
walks the prologue and every tail branch of the wait table (m = S-1, 2, 1, 0 tiles issued after the
awaited one). Each cnt runs with a full last tile and a short one (pieces wholly past the batch), at
a 16-B-aligned and a 4-B-offset base, HdrCalc and HdrVerify, against the oracle (the C restatement
of net_util.c:159-284). One run per case; no repeat-run probes.

(P, H) = (1, 4) is unreachable: a 256-header tile of >= 1-B headers at a stride >= 4 is > 1 KiB.
P is exact for the base's offset in its 16-B line (hdr_pieces), so each case picks its shape for
the lead it runs at.
"""
import numpy as np
import pytest

import netcsum
import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"

INSTANCES = [(p, s, 1) for p in range(1, 6) for s in (2, 3, 4)] + \
            [(p, s, 2) for p in range(1, 7) for s in (2, 3, 4)] + \
            [(p, s, 4) for p in range(2, 7) for s in (2, 3)]


def _pieces(L, st, h, lead):
    return (lead + (64 * h - 1) * st + L + 1023) // 1024


def _shape(P, H, lead):
    """The longest header (len <= stride <= 64, stride a multiple of 4) whose 64H-header tile takes P
    pieces at this lead and that the kernel accepts (hdr_supported, hdr_lanes_h keeps H)."""
    best = None
    for st in range(4, 65, 4):
        for L in range(1, st + 1):
            if _pieces(L, st, 1, lead) > 5 or _pieces(L, st, H, lead) > 6 or _pieces(L, st, H, lead) != P:
                continue
            if best is None or (L, -st) > (best[0], -best[1]):
                best = (L, st)
    return best


@pytest.fixture(autouse=True)
def _tuning():
    def reset():
        netcsum.tune(netcsum.TUNE_KERNEL, 0)
        netcsum.tune(netcsum.TUNE_CHUNKS, 0)
        netcsum.tune(netcsum.TUNE_TILE, -1)
        netcsum.tune(netcsum.TUNE_GRID_BLOCKS, 0)
    reset()
    yield
    reset()


@pytest.mark.parametrize("P,S,H", INSTANCES)
def test_hdr_kernel_every_tail_branch(P, S, H):
    netcsum.tune(netcsum.TUNE_KERNEL, 7)
    netcsum.tune(netcsum.TUNE_CHUNKS, S)
    netcsum.tune(netcsum.TUNE_TILE, H)
    netcsum.tune(netcsum.TUNE_GRID_BLOCKS, 1)
    rng = np.random.default_rng(P * 100 + S * 10 + H)
    TH = 64 * H
    for cnt in range(1, S + 2):
        for short in (0, 5):
            n = 4 * cnt * TH - short
            for lead in (0, 4):
                shape = _shape(P, H, lead)
                if shape is None:
                    continue
                L, st = shape
                host = rng.integers(0, 256, size=lead + n * st + 64, dtype=np.uint8)
                dev = torch.from_numpy(host).to(DEV)
                assert (dev.data_ptr() + lead) % 16 == lead
                for op in (2, 3):
                    out = torch.zeros(n, dtype=torch.int16 if op == 2 else torch.uint8, device=DEV)
                    netcsum.batch_strided(dev[lead:], st, L, None, 0, 0, n, out, op)
                    torch.cuda.synchronize()
                    desc = netcsum.last_launch()
                    assert f"seg_hdr_kernel<P={P},S={S},H={H}>" in desc and "grid=1" in desc, desc
                    got = out.cpu().numpy()
                    got = got.view(np.uint16) if op == 2 else got
                    want = oracle.batch_strided(host, st, L, None, 0, 0, n, op, seg_offset=lead)
                    bad = np.nonzero(got != want)[0]
                    assert bad.size == 0, (cnt, short, lead, op, bad[:5].tolist())
