"""Plan identity the caller controls. The planned batch kinds choose
their form from a plan the previous batch on the same layout sampled on the device, keyed on the
batch's addresses. Two layouts placed alternately at the SAME addresses — the same ring buffer and
stride, the same descriptor arrays — used to run every batch in the other layout's plan. Bound to ids
of their own (NetUtil_MI355X_PlanBind), each keeps its plan; with NETCSUM_TUNE_PLAN_AHEAD 1 even the
first batch of each runs in its plan (a one-block sampler launch the call waits for). Every result is
compared with the oracle.

Rings: 64 Ki frames in 1520-B slots at +14 — A: 1500-B IPv4/TCP datagrams (plan: the whole-span form
0), B: the 40 / 576 / 1500-B mix (plan: live pieces in runs of 32). Pools: 64 Ki TCP segments one per
1520-B buffer at +34 — A: 1480 B each (plan: the live-sector stream, runs of 8), B: 20 / 556 / 1480 B
(runs of 41, the reach)."""
import numpy as np
import pytest

import netcsum
import oracle
import oracle_packets as op

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda"
N = 1 << 16


@pytest.fixture(autouse=True)
def _reset():
    yield
    netcsum.tune(netcsum.TUNE_PLAN_AHEAD, -1)
    netcsum.plan_bind(0)


def _ring_bytes(sizes, slot=1520, lead=14, seed=3):
    """The ring as host bytes: random payload, an IPv4 header + TCP / UDP header per frame (the
    tools/ring_layouts.py shape), checksum fields finalized by the oracle for half the frames."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import ring_layouts
    n = len(sizes)
    rng = np.random.default_rng(seed)
    buf = rng.integers(0, 256, size=n * slot + 256, dtype=np.uint8)
    v = buf[: n * slot].reshape(n, slot)
    v[:, lead:lead + 40] = ring_layouts.headers(np.asarray(sizes, np.int64), seed=seed + 1)
    for i in range(0, n, 4):                          # a quarter of the frames carry valid checksums
        o = i * slot + lead
        q, _ = op.tx_finalize(bytes(buf[o:o + int(sizes[i])]), True)
        buf[o:o + len(q)] = np.frombuffer(q, np.uint8)
    want = np.array([op.rx_validate(bytes(buf[i * slot + lead:(i + 1) * slot])) for i in range(n)], np.uint8)
    return buf, want


def test_ring_layouts_alternating_at_the_same_addresses():
    slot, lead = 1520, 14
    rng = np.random.default_rng(8)
    a_buf, a_want = _ring_bytes(np.full(N, 1500))
    b_buf, b_want = _ring_bytes(np.array([40, 576, 1500])[rng.choice(3, size=N, p=[7 / 12, 4 / 12, 1 / 12])], seed=5)
    d = torch.empty(len(a_buf), dtype=torch.uint8, device=DEV)
    f = torch.zeros(N, dtype=torch.uint8, device=DEV)
    a_h, b_h = torch.from_numpy(a_buf), torch.from_numpy(b_buf)
    layouts = {1: (a_h, a_want, "plan=ring(form0)"), 2: (b_h, b_want, "plan=ring(live)")}

    def run(lid):
        h, want, _ = layouts[lid]
        d.copy_(h)
        netcsum.rx_validate_ipv4(d[lead:], N, f, stride=slot, pkt_len=slot - lead)
        torch.cuda.synchronize()
        got = f.cpu().numpy()
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (lid, netcsum.last_launch(), bad[:5])
        return netcsum.last_launch()

    # addresses alone (id 0, no ahead sampling): each batch runs in the plan the OTHER layout left
    netcsum.tune(netcsum.TUNE_PLAN_AHEAD, 0)
    netcsum.plan_bind(0)
    run(1)
    run(1)
    assert "plan=ring(form0)" in run(2)                # B in A's plan: the stale form (correct, slower)
    assert "plan=ring(live)" in run(1)                 # and A in B's
    # bound to ids, sampled ahead: every batch in its own layout's plan, the first ones included
    netcsum.tune(netcsum.TUNE_PLAN_AHEAD, 1)
    for rep in range(3):
        for lid in (1, 2):
            netcsum.plan_bind(10 + lid)
            desc = run(lid)
            assert layouts[lid][2] in desc, (rep, lid, desc)
            assert ("ahead" in desc) == (rep == 0), (rep, lid, desc)
            if lid == 2:
                assert "pkts_per_wave=32" in desc, desc


def test_pool_layouts_alternating_in_the_same_descriptor_arrays():
    slot, ix = 1520, 34
    rng = np.random.default_rng(9)
    offs = (np.arange(N, dtype=np.int64) * slot + ix)
    a_len = np.full(N, 1480, np.uint16)
    b_len = np.array([20, 556, 1480])[rng.choice(3, size=N, p=[7 / 12, 4 / 12, 1 / 12])].astype(np.uint16)
    buf = rng.integers(0, 256, size=N * slot + 256, dtype=np.uint8)
    ph = rng.integers(0, 256, size=N * 12, dtype=np.uint8)
    base, ph_d = torch.from_numpy(buf).to(DEV), torch.from_numpy(ph).to(DEV)
    off_d = torch.from_numpy(offs).to(DEV)
    len_d = torch.empty(N, dtype=torch.int16, device=DEV)
    out = torch.empty(N, dtype=torch.int16, device=DEV)
    want = {}
    for lid, ln in ((1, a_len), (2, b_len)):
        segs = np.concatenate([buf[o:o + int(m)] for o, m in zip(offs.tolist(), ln.tolist())])
        so = np.zeros(N, np.uint64)
        so[1:] = np.cumsum(ln[:-1].astype(np.uint64))
        want[lid] = (ln, oracle.batch_varlen(segs, so, ln.copy(), ph, 12, 12, oracle.OP_DATA_CALC))
    expect = {1: "segs_per_wave=8 plan=pool(live)", 2: "segs_per_wave=41 plan=pool(live)"}

    def run(lid):
        ln, w = want[lid]
        len_d.copy_(torch.from_numpy(ln.view(np.int16)))
        netcsum.batch_varlen(base, off_d, len_d, ph_d, 12, 12, N, out, netcsum.OP_DATA_CALC)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint16)
        bad = np.nonzero(got != w)[0]
        assert bad.size == 0, (lid, netcsum.last_launch(), bad[:5])
        return netcsum.last_launch()

    netcsum.tune(netcsum.TUNE_PLAN_AHEAD, 0)
    netcsum.plan_bind(0)
    run(1)
    assert expect[1] in run(1)
    assert expect[1] in run(2)                         # the stale plan of the other layout
    netcsum.tune(netcsum.TUNE_PLAN_AHEAD, 1)
    for rep in range(3):
        for lid in (1, 2):
            netcsum.plan_bind(20 + lid)
            desc = run(lid)
            assert expect[lid] in desc, (rep, lid, desc)
            assert ("ahead" in desc) == (rep == 0), (rep, lid, desc)
