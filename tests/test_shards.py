"""Sharding and the cross-rank hit gather, world_size 2 over gloo on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from patmatchdocker_amd import shards


def test_shard_range_covers_records():
    for n, w in [(10, 3), (7, 8), (1000, 8), (5, 1)]:
        got = [shards.shard_range(n, w, r) for r in range(w)]
        assert sum(c for _, c in got) == n
        assert all(got[i][0] + got[i][1] == got[i + 1][0] for i in range(w - 1))
        assert got[0][0] == 0


def test_to_global_keeps_pattern_field():
    keys = torch.tensor([(1 << 48) | 5, (0 << 48) | 7], dtype=torch.int64)
    out = shards.to_global(keys, 1000)
    assert (out >> 48).tolist() == [1, 0]
    assert (out & shards.POS_MASK).tolist() == [1005, 1007]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank r owns positions [r*1000, r*1000+1000); two patterns, uneven counts
        g = torch.Generator().manual_seed(rank)
        n = 3 + 4 * rank
        pos = torch.randint(0, 1000, (n,), generator=g) 
        pat = torch.randint(0, 3, (n,), generator=g)
        keys = (pat << 48) | pos
        order = torch.argsort(keys)
        keys, lens = keys[order], torch.full((n,), 15, dtype=torch.int32)
        out = shards.gather_hits(shards.to_global(keys, rank * 1000), lens)
        if rank == 0:
            results.put((out[0].tolist(), out[1].tolist()))
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [2, 4])
def test_gather_ranks_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    keys, lens = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # expected: union of both ranks' keys shifted by rank*1000, globally sorted
    want = []
    for rank in range(world):
        g = torch.Generator().manual_seed(rank)
        n = 3 + 4 * rank
        pos = torch.randint(0, 1000, (n,), generator=g)
        pat = torch.randint(0, 3, (n,), generator=g)
        want += (((pat << 48) | pos) + rank * 1000).tolist()
    assert keys == sorted(want)
    assert lens == [15] * len(want)
