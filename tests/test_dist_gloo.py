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
