"""Multi-process (world_size 2, gloo, CPU) check of bench.py's sharding: each rank owns a
contiguous slice of ONE global synthetic batch (bytes = matching slice of the global splitmix64
stream, pseudo-headers from the global index), computes its checksums independently (no data-path
collective), and the union over ranks equals a single-process run over the whole batch. Also the
max-over-ranks reduction bench.py applies to the timed region.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, L, plen, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, cnt = bench.shard_range(rank, n)
    seg, ph = bench.host_c2_shard(oracle, start, cnt, L, plen)
    out = oracle.batch_strided(seg, L, L, ph, plen, plen, cnt, oracle.OP_DATA_CALC)
    t = torch.from_numpy(out.astype(np.int32))
    gathered = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(gathered, t)
    wall = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((torch.cat(gathered).numpy().astype(np.uint16), float(wall.item())))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_shards_union_equals_single_run(world):
    n, L, plen = 1500, 1500, 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, L, plen, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, wall = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seg, ph = bench.host_c2_shard(oracle, 0, world * n, L, plen)
    want = oracle.batch_strided(seg, L, L, ph, plen, plen, world * n, oracle.OP_DATA_CALC)
    assert np.array_equal(got, want)
    assert wall == 0.5 + (world - 1)


def test_shard_ranges_partition_the_batch():
    for world in (1, 2, 4, 8):
        n = 1 << 20
        ranges = [bench.shard_range(r, n) for r in range(world)]
        assert ranges[0][0] == 0
        for (s0, c0), (s1, _) in zip(ranges, ranges[1:]):
            assert s0 + c0 == s1
        assert sum(c for _, c in ranges) == world * n


def test_pseudo_headers_shape_and_fields():
    ph = bench.c2_pseudo_headers(5, 3, 1500, 12).reshape(3, 12)
    assert (ph[:, 9] == 6).all() and (ph[:, 8] == 0).all()
    assert ph[0, 10] == 1500 >> 8 and ph[0, 11] == 1500 & 0xFF
    assert bytes(ph[0, 0:4]) == bytes([0x0A, 0, 0, 5])


def _varlen_worker(rank, world, port, lens, q):
    """Rank r checksums ITS byte-balanced range of one global C4-shaped batch (contiguous, packed)."""
    import netcsum
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first = netcsum.shard_varlen(lens, 12, world)
    base, off, ph = _c4_host(lens)
    a, b = int(first[rank]), int(first[rank + 1])
    out = oracle.batch_varlen(base, off[a:b], lens[a:b], ph[12 * a:12 * b], 12, 12, oracle.OP_DATA_CALC)
    mine = torch.from_numpy(out.astype(np.int32))
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([b - a]))
    m = max(int(s.item()) for s in sizes)
    parts = [torch.zeros(m, dtype=torch.int32) for _ in sizes]
    dist.all_gather(parts, torch.nn.functional.pad(mine, (0, m - mine.numel())))   # test-only gather
    parts = [p[: int(s.item())] for p, s in zip(parts, sizes)]
    byte_tot = torch.tensor([int(lens[a:b].astype(np.int64).sum()) + 12 * (b - a)])
    allb = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allb, byte_tot)
    if rank == 0:
        q.put((torch.cat(parts).numpy().astype(np.uint16), [int(x.item()) for x in allb]))
    dist.destroy_process_group()


def _c4_host(lens):
    off = np.zeros(len(lens), np.uint64)
    off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    base = oracle.fill(0, int(off[-1]) + int(lens[-1]) + 16, bench.SEED, 0)
    ph = np.random.default_rng(11).integers(0, 256, size=12 * len(lens), dtype=np.uint8)
    return base, off, ph


def test_varlen_byte_balanced_shards_union_equals_single_run():
    """C4 split for N GPUs: NetUtil_MI355X_ShardVarLen's prefix-sum ranges carry equal
    bytes to within one datagram and their union is the single-GPU result."""
    world = 2
    lens = np.random.default_rng(7).integers(40, 9001, size=3000).astype(np.uint16)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_varlen_worker, args=(r, world, port, lens, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, byte_tot = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    base, off, ph = _c4_host(lens)
    want = oracle.batch_varlen(base, off, lens, ph, 12, 12, oracle.OP_DATA_CALC)
    assert np.array_equal(got, want)
    assert max(byte_tot) - min(byte_tot) <= 2 * (9000 + 12)


def test_varlen_shard_boundaries():
    import netcsum
    rng = np.random.default_rng(7)
    lens = rng.integers(40, 9001, size=1 << 20).astype(np.uint16)
    for world in (1, 2, 3, 4, 8):
        f = netcsum.shard_varlen(lens, 12, world)
        assert f[0] == 0 and f[-1] == len(lens) and (np.diff(f.astype(np.int64)) >= 0).all()
        b = [int(lens[f[r]:f[r + 1]].astype(np.int64).sum()) + 12 * int(f[r + 1] - f[r]) for r in range(world)]
        assert max(b) - min(b) <= 2 * (9000 + 12), (world, b)
    assert list(netcsum.shard_varlen(np.zeros(0, np.uint16), 12, 4)) == [0, 0, 0, 0, 0]
    assert list(netcsum.shard_varlen(np.array([100], np.uint16), 0, 3)) == [0, 1, 1, 1]


def _rank_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank 1 is the slow device: a longer wall time, a lower fraction of its own read ceiling
    own = {"rank": rank, "local_rank": rank, "device": rank, "wall_s": 0.10 + 0.02 * rank, "kernel_ms": 3.5 + 0.3 * rank,
           "per_gpu_GiBps": 6700.0 - 500.0 * rank, "run_stream_read_probe_GBps": 7300.0,
           "read_stream_probe_GBps": 6990.0, "frac_of_run_stream_read_probe": 0.98 - 0.07 * rank,
           "parity_sample_ok": 1.0}
    recs = bench.rank_records(dist, "cpu", own, world)
    if rank == 0:
        q.put(bench.rank_summary(recs))
    dist.destroy_process_group()


def test_rank_records_name_the_slowest_device():
    """bench.py at N > 1: every rank's own per-GPU rate, kernel time and read
    ceilings are all-gathered, and rank 0's line names the slowest rank and its LOCAL_RANK."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    summ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r["rank"] for r in summ["per_rank"]] == [0, 1]
    assert summ["slowest_rank"] == 1 and summ["slowest_local_rank"] == 1 and summ["fastest_rank"] == 0
    assert summ["min_per_gpu"] == 6200.0 and summ["max_per_gpu"] == 6700.0
    assert summ["spread_max_over_min"] == round(6700.0 / 6200.0, 4)
    assert summ["min_frac_of_run_stream_read_probe"] == 0.91
    assert summ["per_rank"][1]["kernel_ms"] == 3.8 and all(r["parity_sample_ok"] for r in summ["per_rank"])
    assert set(summ["per_rank"][0]) >= {"per_gpu_GiBps", "wall_s", "run_stream_read_probe_GBps", "local_rank"}
